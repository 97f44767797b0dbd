"use strict";
/**
 * fmt.js — JavaScript batch replay driver over the N-API addon (../fmt_napi.node → libfmt.so).
 *
 * This is the host side a Fluid runtime calls. It mirrors the reference's DDS message surface:
 *   SharedObjectCore.processMessagesCore(messagesCollection)   shared-object-base/src/sharedObject.ts:415
 *   IRuntimeMessageCollection {envelope, local, messagesContent}  runtime-definitions/src/protocol.ts:80-142
 *   SharedSegmentSequence.processMessage rebuilds each message as {...envelope, contents,
 *     clientSequenceNumber}                                     sequence/src/sequence.ts:873-919
 *   SharedMap.processMessagesCore → MapKernel.tryProcessMessage  map/src/map.ts:288-311, mapKernel.ts:619
 * Instead of applying every message on the JS thread, messages of many documents are packed into
 * the flat records of include/fmt.h (exactly as fluidframework_amd/streams.py packs them; the CPU
 * test suite checks the two packers byte for byte) and replayed on the GPU in one async call.
 *
 * Written for the Node in this image (v12): CommonJS, no `??` / `?.`.
 */
const path = require("path");
const summary = require("./summary.js");

const MT_INSERT = 0, MT_REMOVE = 1, MT_ANNOTATE = 2, MT_GROUP = 3, MT_OBLITERATE = 4, MT_OBLITERATE_SIDED = 5; // ops.ts:61-71
const MAP_SET = 0, MAP_DELETE = 1, MAP_CLEAR = 2, MAP_KIND_SHIFT = 30;
const MAP_VALUE_UNDEFINED = 0x3fffffff, MAP_ABSENT = 0xffffffff;
const MAP_EV_SUBMIT = 0, MAP_EV_ACK = 1, MAP_EV_ROLLBACK = 2;  // fmt.h FMT_MAP_EV_*
const FMT_MT_F_GROUP_CONT = 1, FMT_MT_F_CATCHUP = 2, FMT_MT_F_RMORDER = 4;
const FMT_MT_F_START_BEFORE = 8, FMT_MT_F_END_BEFORE = 16; // sided obliterate places (client.ts:680-700)
const FMT_MT_F_MARKER = 32, FMT_MT_SEG_MARKER = 0x80000000, FMT_MT_LEAF_MARKER = 0x8000; // Marker segments
// legacy relativePos1/2 (ops.ts IRelativePosition): pos1/pos2 index the relpos table (fmt_mt_relpos, 16 B)
const FMT_MT_F_LOADSEG = 256, FMT_MT_CLIENT_NONCOLLAB = 0xfe; // SnapshotV1 body segments with merge info
const FMT_MT_F_LEN_HI_MASK = 0x00ff0000; // insert length bits 16..23 (fmt.h FMT_MT_F_LEN_HI_SHIFT)
const FMT_MT_F_REL1 = 64, FMT_MT_F_REL2 = 128, FMT_MT_NO_MARKER = 0xffffffff, FMT_MT_REL_BEFORE = 1;
const MARKER_ID_KEY = "markerId"; // reservedMarkerIdKey
// annotate-adjust (fmt.h): props_kv escape, computed value ids, fmt_mt_adjust flags
const FMT_MT_VALUE_ADJUST = 0xffff, FMT_MT_VALUE_COMPUTED = 0x8000;
const FMT_MT_ADJ_MIN = 1, FMT_MT_ADJ_MIN_NULL = 2, FMT_MT_ADJ_MAX = 4, FMT_MT_ADJ_MAX_NULL = 8;
const FMT_NON_COLLAB_CLIENT = -2; // fmt.h: the insert client of a segment without merge info
// f4, the local client (fmt.h): a submission, the ack of the oldest pending op, rollback of the newest,
// reconnect (regeneratePendingOp for every pending op)
const FMT_MT_F_LOCAL = 512, FMT_MT_F_ACK = 1024, FMT_MT_F_ROLLBACK = 2048, FMT_MT_F_REGEN = 4096;

/** The refType of a Marker spec {marker: {refType}, props?} (IJSONMarkerSegment), or null. */
function markerRefType(spec) {
	if (!(spec && typeof spec === "object" && "marker" in spec)) return null;
	if (!Object.keys(spec).every((k) => k === "marker" || k === "props") || !spec.marker || typeof spec.marker !== "object") {
		throw new UnsupportedOp("marker spec");
	}
	const r = spec.marker.refType;
	if (!Number.isInteger(r) || r < 0 || r > 0xffff) throw new UnsupportedOp("marker refType");
	return r;
}
const MAX_CLIENTS = 253; // small tier 31 writers, large 63, huge 253 (streams.py; 0xFE names NonCollab)
const RECYCLE_FROM = 32; // fresh short ids up to the small tier's 31 writers, then recycled (streams.py)
const NOT_REMOVED = 0x7fffffff;
const MT_OP_BYTES = 32, MAP_OP_BYTES = 16, LEAF_BYTES = 32, DOC_RESULT_BYTES = 48, PROPSET_BYTES = 36;
const CATCHUP_BYTES = 16, SNAPSHOT_DOC_BYTES = 32;
const NO_PROPS = 0xffffffff;
const PROPS_MAX = 8, FMT_MT_PROPS_CONT = 0xffffffff; // fmt.h: entries per prop-set record; n of a continuation record

let addon = null;
/** The native addon; throws if it was not built (there is no JavaScript fallback engine). */
function native() {
	if (addon === null) {
		addon = require(path.join(__dirname, "..", "fmt_napi.node"));
	}
	return addon;
}

class UnsupportedOp extends Error {
	constructor(msg) {
		super(msg);
		this.code = "FMT_E_UNSUPPORTED";
	}
}

/** Interns strings to dense ids, first come first served. */
class Dictionary {
	constructor(reserved) {
		this.items = reserved ? reserved.slice() : [];
		this.ids = new Map();
		this.items.forEach((s, i) => this.ids.set(s, i));
	}
	intern(s) {
		let i = this.ids.get(s);
		if (i === undefined) {
			i = this.items.length;
			this.items.push(s);
			this.ids.set(s, i);
		}
		return i;
	}
}

/** Growable byte buffer of fixed-size records. */
class RecordBuffer {
	constructor(recordBytes) {
		this.rb = recordBytes;
		this.buf = new ArrayBuffer(recordBytes * 1024);
		this.view = new DataView(this.buf);
		this.n = 0;
	}
	next() {
		if ((this.n + 1) * this.rb > this.buf.byteLength) {
			const nb = new ArrayBuffer(this.buf.byteLength * 2);
			new Uint8Array(nb).set(new Uint8Array(this.buf));
			this.buf = nb;
			this.view = new DataView(nb);
		}
		return this.n++ * this.rb;
	}
	bytes() {
		return new Uint8Array(this.buf, 0, this.n * this.rb).slice();
	}
}

class U16Arena {
	constructor() {
		this.a = new Uint16Array(4096);
		this.n = 0;
	}
	push(s) {
		const off = this.n;
		if (this.n + s.length > this.a.length) {
			let cap = this.a.length * 2;
			while (cap < this.n + s.length) cap *= 2;
			const na = new Uint16Array(cap);
			na.set(this.a.subarray(0, this.n));
			this.a = na;
		}
		for (let i = 0; i < s.length; i++) this.a[this.n + i] = s.charCodeAt(i); // UTF-16 code units
		this.n += s.length;
		return [off, s.length];
	}
	finish() {
		return this.a.slice(0, this.n);
	}
}

/** Per-document packing state: short client ids (client.ts:831-855, observer = 0). */
class MergeTreeDocBuilder {
	constructor(owner, index, observer) {
		this.owner = owner;
		this.index = index;
		this.clientIds = new Map([[observer, 0]]);
		this.clientNames = [observer];
		this.lastStamp = [null]; // per short id: the current holder's latest stamp seq
		this.minSeq = 0; // the engine's minSeq when the next message applies
		this.nOps = 0;
		this.messages = []; // {message, firstOp, count} when the builder keeps messages
		// idToMarker history (streams.py _DocBuilder): exact while every marker id names one marker
		// and no annotate rewrites an id
		this.markerIds = new Set();
		this.markerAmbiguous = false;
		this.usesRelpos = false;
		// f4: the document's observer is a local client with events of its own (streams.py _DocBuilder)
		this.local = false;
		this.pending = []; // [type, payload, refSeq] of each pending local op, oldest first
		this.regenRef = 0;
		this.curSeq = 0; // the last message's seq: a local op's refSeq (sequence.ts:666 currentRefSeq)
	}
	noteMarkerId(props) {
		const mid = props ? props[MARKER_ID_KEY] : undefined;
		if (mid) {
			const k = JSON.stringify(mid);
			if (this.markerIds.has(k)) this.markerAmbiguous = true;
			this.markerIds.add(k);
			this.checkMarkers();
		}
	}
	checkMarkers() {
		if (this.usesRelpos && this.markerAmbiguous) {
			throw new UnsupportedOp("relative positions in a document whose marker ids repeat or are re-annotated");
		}
	}
	noteOp(op) {
		if (op === null) return;
		if (op.type === MT_INSERT && markerRefType(op.seg) !== null) this.noteMarkerId(op.seg.props);
		if (op.type === MT_ANNOTATE && op.props && Object.prototype.hasOwnProperty.call(op.props, MARKER_ID_KEY)) this.markerAmbiguous = true;
		const none = (v) => v === undefined || v === null;
		if ((none(op.pos1) && !none(op.relativePos1)) || (none(op.pos2) && !none(op.relativePos2))) this.usesRelpos = true;
		this.checkMarkers();
	}
	/**
	 * getOrAddShortClientId (client.ts:831-855) with recycling (mirrors streams.py short_client): a
	 * new client takes, past RECYCLE_FROM - 1 ids, the id of a client whose every stamp is at or
	 * below the engine's minSeq; `seq` notes a stamp of the client.
	 */
	shortClient(longId, seq) {
		const id = longId === null || longId === undefined ? "server" : longId;
		let i = this.clientIds.get(id);
		if (i === undefined) {
			i = this.clientNames.length;
			if (i >= RECYCLE_FROM) {
				// the engine's minSeq: in a document with local events it is also bounded by the oldest
				// pending op's refSeq (getMinInFlightRefSeq, client.ts:1374-1378)
				let floor = this.minSeq;
				for (const p of this.pending) if (p[2] < floor) floor = p[2];
				for (let j = 1; j < this.clientNames.length; j++) {
					const st = this.lastStamp[j];
					if (st === null || st <= floor) {
						this.clientIds.delete(this.clientNames[j]);
						this.clientNames[j] = id;
						this.lastStamp[j] = null;
						i = j;
						break;
					}
				}
			}
			if (i === this.clientNames.length) {
				if (i > MAX_CLIENTS) throw new UnsupportedOp(`more than ${MAX_CLIENTS} clients with stamps above minSeq in one document`);
				this.clientNames.push(id);
				this.lastStamp.push(null);
			}
			this.clientIds.set(id, i);
		}
		if (seq !== undefined && (this.lastStamp[i] === null || seq > this.lastStamp[i])) this.lastStamp[i] = seq;
		return i;
	}
	/** One ISequencedDocumentMessage with merge-tree contents (client.applyMsg, client.ts:1358). */
	addMessage(msg) {
		if (this.owner.current !== this) {
			throw new UnsupportedOp("documents must be packed contiguously (finish one before the next)");
		}
		const client = this.shortClient(msg.clientId, msg.sequenceNumber);
		const contents = msg.contents;
		let members = contents.type === MT_GROUP ? contents.ops : [contents];
		if (members.length === 0) members = [null]; // empty group: only advances the window
		// a message of the local client itself acknowledges its oldest pending ops, one per member
		// (client.ts:1367-1368 ackPendingSegment)
		const ack = this.local && client === 0;
		if (this.owner.keepMessages) this.messages.push({ message: msg, firstOp: this.nOps, count: members.length });
		members.forEach((op, k) => {
			if (!ack) this.noteOp(op); // (an ack repeats the local op noted at its submission)
			let flags = k > 0 ? FMT_MT_F_GROUP_CONT : 0;
			if (ack) {
				if (op === null || this.pending.length === 0 || this.pending[0][0] !== op.type) {
					throw new Error("an ack that is not the oldest pending local op"); // mergeTree.ts:1331-1340
				}
				this.pending.shift();
				flags |= FMT_MT_F_ACK;
			}
			this.owner.packOp(op, msg.sequenceNumber, msg.referenceSequenceNumber,
				msg.minimumSequenceNumber, client, flags);
			this.nOps++;
		});
		if (msg.minimumSequenceNumber > this.minSeq) this.minSeq = msg.minimumSequenceNumber; // updateSeqNumbers
		this.curSeq = msg.sequenceNumber;
	}
	/**
	 * A local submission (insertSegmentLocal / removeRangeLocal / annotateRangeLocal,
	 * client.ts:273-355): op contents with positions in the local view; a GROUP op
	 * (localTransaction, client.ts:1600-1629) submits its members one by one. Mirrors streams.py.
	 */
	localOp(op) {
		if (this.owner.current !== this) throw new UnsupportedOp("documents must be packed contiguously (finish one before the next)");
		const members = op.type === MT_GROUP ? op.ops : [op];
		for (const m of members) {
			if (m.type !== MT_INSERT && m.type !== MT_REMOVE && m.type !== MT_ANNOTATE) throw new UnsupportedOp("local obliterate");
			const none = (v) => v === undefined || v === null;
			if ((none(m.pos1) && !none(m.relativePos1)) || (m.type !== MT_INSERT && none(m.pos2) && !none(m.relativePos2))) {
				throw new UnsupportedOp("local op with relative positions");
			}
			this.noteOp(m);
			this.owner.packOp(m, 0, this.curSeq, 0, 0, FMT_MT_F_LOCAL);
			const o = (this.owner.ops.n - 1) * MT_OP_BYTES;
			this.local = true;
			this.pending.push([m.type, this.owner.ops.view.getUint32(o + 20, true), this.curSeq]);
			this.nOps++;
		}
	}
	/** Rollback of the newest pending op (client.ts:554; a GROUP op: once per member). */
	localRollback() {
		if (this.pending.length === 0) throw new Error("rollback without a pending local op");
		const [t, payload] = this.pending.pop(); // (refSeq dropped)
		this.owner.rawOp(0, 0, 0, 0, 0, payload, 0, 0, t, FMT_MT_F_ROLLBACK);
		this.nOps++;
	}
	/**
	 * Reconnect: regeneratePendingOp for every pending op (client.ts:1452-1542). The ops it returns
	 * (MergeTreeReplay.regenerated) become the pending ops whose acks follow: pass them here or to
	 * regenPending once known.
	 */
	localRegen(newOps, newClientId) {
		// newClientId: the new connection's clientId keeps short id 0 (startOrUpdateCollaboration,
		// client.ts:1719-1725; the old long id stays mapped too), so the resubmitted ops come back as acks
		if (newClientId !== undefined && newClientId !== null) this.renameLocal(newClientId);
		this.local = true;
		this.owner.rawOp(0, 0, 0, 0, 0, 0, 0, 0, 0, FMT_MT_F_REGEN);
		this.nOps++;
		// a resubmitted op keeps its original refSeq (sequence.ts:782-790): the oldest of the old pending
		// ops' refSeqs still bounds the engine's minSeq
		this.regenRef = this.pending.reduce((m, p) => Math.min(m, p[2]), this.curSeq);
		this.pending = [];
		if (newOps) this.regenPending(newOps);
	}
	/** startOrUpdateCollaboration with a new long id (client.ts:1719-1725): it names short id 0 now. */
	renameLocal(newClientId) {
		const i = this.clientIds.get(newClientId);
		if (i !== undefined && i !== 0) throw new UnsupportedOp("a reconnect clientId that already names another client");
		this.clientIds.set(newClientId, 0);
		this.clientNames[0] = newClientId;
	}
	regenPending(newOps) {
		this.pending = newOps.map((op) => [op.type, op.type === MT_ANNOTATE ? this.owner.propsOp(op.props || {}, op.adjust) : 0, this.regenRef]);
	}
	/**
	 * SharedObjectCore.processMessagesCore shape: a bunch sharing one envelope (sequence.ts:873-919).
	 * A local bunch (the client's own messages coming back sequenced) acknowledges its pending ops.
	 */
	processMessagesCore(messagesCollection) {
		const { envelope, messagesContent } = messagesCollection;
		if (messagesCollection.local && (!this.local || this.clientIds.get(envelope.clientId) !== 0)) {
			throw new UnsupportedOp("a local bunch from a client other than the document's observer, or with no pending local ops");
		}
		for (const mc of messagesContent) {
			this.addMessage(Object.assign({}, envelope, {
				contents: mc.contents,
				clientSequenceNumber: mc.clientSequenceNumber,
			}));
		}
	}
}

/** JS object key order (OrdinaryOwnPropertyKeys): Object.keys already yields it. */
function jsKeyOrder(obj) {
	return Object.keys(obj);
}

/** Packs many documents' sequenced merge-tree messages (mirror of streams.py MergeTreeStreamBuilder). */
class MergeTreeStreamBuilder {
	/**
	 * @param options - {keepMessages}: keep each document's messages (as applyMsg received them)
	 * for the legacy summary's catch-up blob.
	 */
	constructor(options) {
		this.keepMessages = !!(options && options.keepMessages);
		this.keys = new Dictionary();
		this.values = new Dictionary(["null"]);
		this.text = new U16Arena();
		this.ops = new RecordBuffer(MT_OP_BYTES);
		this.propsOps = new Map();
		this.propsList = [];
		this.docs = [];
		this.docInit = [];
		this.snapshots = []; // per doc: null or [firstSeg, nHeader, nBody, minSeq, seq]
		this.snapshotSegs = []; // [textOff, len, propsOp]
		this.segDoc = []; // per snapshot segment: its document
		this.relpos = []; // [marker value id, offset, flags]
		this.snapshotInfo = []; // per snapshot segment: [insSeq, insClient, rmFirst, rmCount] (V1 merge info)
		this.snapshotStamps = []; // [seq, client, kind]
		this.hasMergeInfo = false;
		this.adjusts = []; // fmt_mt_adjust rows [delta, min, max, flags]
		this.adjustRows = new Map();
		this.current = null;
	}
	beginDoc(initialText, observer) {
		const d = new MergeTreeDocBuilder(this, this.docs.length, observer === undefined ? "A" : observer);
		this.docs.push(d);
		this.docInit.push(initialText ? this.text.push(initialText) : [0, 0]);
		this.snapshots.push(null);
		this.current = d;
		return d;
	}
	/** specToSegment for a text spec: "text" or {text, props} (IJSONTextSegment). */
	specToSeg(spec) {
		let text, props;
		const rtype = markerRefType(spec);
		if (rtype !== null) {
			const [off] = this.text.push(String.fromCharCode(rtype));
			const p = spec.props;
			this.snapshotSegs.push([off, (1 | FMT_MT_SEG_MARKER) >>> 0, p && Object.keys(p).length ? this.propsOp(p) : NO_PROPS]);
			this.segDoc.push(this.docs.length);
			return;
		}
		if (typeof spec === "string") {
			text = spec;
		} else if (spec && typeof spec === "object" && typeof spec.text === "string" &&
			Object.keys(spec).every((k) => k === "text" || k === "props")) {
			text = spec.text;
			props = spec.props;
		} else {
			throw new UnsupportedOp("markers and segments with merge info (SnapshotV1) are not loaded");
		}
		if (text.length === 0) throw new Error("empty segment in a summary chunk");
		const [off, len] = this.text.push(text);
		this.snapshotSegs.push([off, len, props && Object.keys(props).length ? this.propsOp(props) : NO_PROPS]);
		this.segDoc.push(this.docs.length);
	}
	/**
	 * specToSegment's stamps for a V1 segment with merge info (snapshotLoader.ts:105-175): insert
	 * {seq ?? 0, client ?? NonCollabClient}; setRemove stamps at removedSeq per removedClientIds entry
	 * (removedClient alone in the back-compat format); sliceRemove stamps movedSeqs[i] /
	 * movedClientIds[i]; sorted by seq (stable). Mirrors streams.py _merge_info.
	 */
	mergeInfo(spec, d) {
		this.hasMergeInfo = true;
		const insSeq = spec.seq === undefined ? 0 : spec.seq;
		const insClient = spec.client === undefined || spec.client === null ? FMT_NON_COLLAB_CLIENT : d.shortClient(spec.client, insSeq);
		const stamps = [];
		if (spec.removedSeq !== undefined) {
			let ids = spec.removedClientIds;
			if (ids === undefined && spec.removedClient !== undefined) ids = [spec.removedClient];
			if (ids === undefined) throw new Error("must have removedClient ids");
			for (const c of ids) stamps.push([spec.removedSeq, d.shortClient(c, spec.removedSeq), 0]);
		}
		if (spec.movedSeq !== undefined) {
			const seqs = spec.movedSeqs, ids = spec.movedClientIds;
			if (seqs === undefined || ids === undefined || seqs.length !== ids.length) throw new Error("must have movedIds ids");
			seqs.forEach((s, i) => stamps.push([s, d.shortClient(ids[i], s), 1]));
		}
		const sorted = stamps.map((x, i) => [x, i]).sort((a, b) => a[0][0] - b[0][0] || a[1] - b[1]).map((x) => x[0]);
		const first = this.snapshotStamps.length;
		for (const x of sorted) this.snapshotStamps.push(x);
		return [insSeq, insClient, first, sorted.length];
	}
	/**
	 * A document that starts from a SharedString summary (SnapshotLoader, snapshotLoader.ts:59-348):
	 * a legacy header + optional body, or SnapshotV1's header + body_0, body_1, ... (pass the bodies
	 * as an array), and optionally the legacy catchupOps blob, whose messages become the first ops
	 * after loadCore's validation (sequence.ts:818-863). V1 header segments with merge info keep
	 * their stamps; when any segment has merge info, the body-chunk segments become
	 * FMT_MT_F_LOADSEG inserts ahead of the messages (loadBody appends each through insertSegments
	 * at the local length, snapshotLoader.ts:254-309; mirrors streams.py).
	 */
	beginDocFromSummary(header, body, catchupOps, observer) {
		const h = JSON.parse(header);
		const md = h.headerMetadata;
		if (md === undefined) throw new Error("header metadata not available");
		const chunks = [h];
		if (body !== undefined && body !== null) for (const b of Array.isArray(body) ? body : [body]) chunks.push(JSON.parse(b));
		if (md.orderedChunkMetadata.length !== chunks.length) {
			throw new Error("summary chunks do not match headerMetadata.orderedChunkMetadata");
		}
		const specsOf = (c) => (c.version === "1" ? c.segments : c.segmentTexts);
		const d = new MergeTreeDocBuilder(this, this.docs.length, observer === undefined ? "snapshot" : observer);
		d.minSeq = md.minSequenceNumber === undefined ? md.sequenceNumber : md.minSequenceNumber;
		d.curSeq = md.sequenceNumber;
		const first = this.snapshotSegs.length;
		let anyInfo = false;
		chunks.forEach((c) => {
			for (let spec of specsOf(c)) {
				let info = [0, FMT_NON_COLLAB_CLIENT, 0, 0];
				if (spec && typeof spec === "object" && "json" in spec) { // hasMergeInfo
					anyInfo = true;
					info = this.mergeInfo(spec, d);
					spec = spec.json;
				}
				if (markerRefType(spec) !== null) d.noteMarkerId(spec.props); // loaded markers register their ids too
				this.specToSeg(spec);
				this.snapshotInfo.push(info);
			}
		});
		const nHeader = specsOf(h).length;
		let nBody = this.snapshotSegs.length - first - nHeader;
		if (nHeader + nBody !== md.totalSegmentCount) throw new Error("Mismatch in totalSegmentCount");
		const seq = md.sequenceNumber;
		const minSeq = md.minSequenceNumber === undefined ? seq : md.minSequenceNumber;
		this.docs.push(d);
		this.docInit.push([0, 0]);
		this.current = d;
		if (anyInfo && nBody > 0) {
			// each body segment: an insert at the local length from PriorPerspective(0, its client), a run
			// of segments without merge info in one insertSegments call (FMT_MT_F_GROUP_CONT)
			// flushBatch (snapshotLoader.ts:291-296) never clears its batch: a segment without merge info
			// before one with merge info gets inserted again by every later flush, so that shape is refused
			let universalSeen = false;
			for (let k = first + nHeader; k < first + nHeader + nBody; k++) {
				const [insSeq, insClient] = this.snapshotInfo[k];
				const universal = insClient === FMT_NON_COLLAB_CLIENT && insSeq === 0;
				if (universalSeen && !universal) {
					throw new UnsupportedOp("a SnapshotV1 body where a segment without merge info precedes one with " +
						"merge info (the reference's loadBody re-inserts the batched segments)");
				}
				universalSeen = universalSeen || universal;
			}
			let prevUniversal = false;
			for (let k = first + nHeader; k < first + nHeader + nBody; k++) {
				const [off, ln, pid] = this.snapshotSegs[k];
				const [insSeq, insClient] = this.snapshotInfo[k];
				const universal = insClient === FMT_NON_COLLAB_CLIENT && insSeq === 0;
				const nUnits = (ln & ~FMT_MT_SEG_MARKER) >>> 0;
				let flags = FMT_MT_F_LOADSEG | ((ln & FMT_MT_SEG_MARKER) ? FMT_MT_F_MARKER : 0) |
					(nUnits & FMT_MT_F_LEN_HI_MASK);
				if (universal && prevUniversal) flags |= FMT_MT_F_GROUP_CONT;
				prevUniversal = universal;
				if (nUnits > 0xffffff) throw new UnsupportedOp("a SnapshotV1 body segment longer than 2^24 - 1 UTF-16 units");
				const o = this.ops.next();
				const v = this.ops.view;
				v.setInt32(o + 0, insSeq, true);
				v.setInt32(o + 4, 0, true);
				v.setInt32(o + 8, minSeq, true);
				v.setInt32(o + 12, k, true);
				v.setInt32(o + 16, pid !== NO_PROPS ? pid + 1 : 0, true);
				v.setUint32(o + 20, off, true);
				v.setUint16(o + 24, nUnits & 0xffff, true);
				v.setUint8(o + 26, insClient === FMT_NON_COLLAB_CLIENT ? FMT_MT_CLIENT_NONCOLLAB : insClient);
				v.setUint8(o + 27, MT_INSERT);
				v.setUint32(o + 28, flags, true);
				d.nOps++;
			}
			nBody = 0; // the document loads its header alone
		}
		this.snapshots.push([first, nHeader, nBody, minSeq, seq]);
		if (catchupOps !== undefined && catchupOps !== null) {
			let cur = seq;
			for (const m of JSON.parse(catchupOps)) {
				if (m.minimumSequenceNumber < minSeq || m.referenceSequenceNumber < minSeq ||
					m.sequenceNumber <= minSeq || m.sequenceNumber < cur) {
					throw new Error("Invalid catchup operations in snapshot");
				}
				cur = m.sequenceNumber;
				d.addMessage(m);
			}
		}
		return d;
	}
	/** An AdjustParams {delta, min?, max?} (ops.ts:191-208) as an fmt_mt_adjust row (streams.py _adjust_row). */
	adjustRow(params) {
		if (!params || typeof params !== "object" || !("delta" in params)) throw new UnsupportedOp("adjust without a delta");
		const num = (v) => {
			if (v === null) return null;
			if (typeof v !== "number") throw new UnsupportedOp("non-numeric adjust parameter");
			return v;
		};
		const delta = num(params.delta);
		let flags = 0, lo = 0, hi = 0;
		if ("min" in params) {
			flags |= FMT_MT_ADJ_MIN | (params.min === null ? FMT_MT_ADJ_MIN_NULL : 0);
			lo = num(params.min) || 0;
		}
		if ("max" in params) {
			flags |= FMT_MT_ADJ_MAX | (params.max === null ? FMT_MT_ADJ_MAX_NULL : 0);
			hi = num(params.max) || 0;
		}
		const row = [delta === null ? 0 : delta, lo, hi, flags];
		const k = row.join(",");
		let i = this.adjustRows.get(k);
		if (i === undefined) {
			i = this.adjusts.length;
			this.adjustRows.set(k, i);
			this.adjusts.push(row);
		}
		return i;
	}
	/** Raw (key, value) changes in key order, then adjust changes (opToChanges,
	 * segmentPropertiesManager.ts:86-95), held as [key, value id] / [key, -1, adjust row] over the
	 * batch-wide value dictionary; finish() packs them with batch-global or document-local value ids
	 * (streams.py _props_op). */
	propsOp(props, adjust) {
		const kv = [];
		for (const k of jsKeyOrder(props)) {
			const v = props[k];
			const keyId = this.keys.intern(k);
			if (keyId > 0xffff) throw new UnsupportedOp("more than 65536 distinct property keys in a batch");
			kv.push([keyId, v === null ? 0 : this.values.intern(JSON.stringify(v))]);
		}
		for (const k of jsKeyOrder(adjust || {})) {
			const keyId = this.keys.intern(k);
			if (keyId > 0xffff) throw new UnsupportedOp("more than 65536 distinct property keys in a batch");
			kv.push([keyId, -1, this.adjustRow(adjust[k])]);
		}
		const t = kv.map((e) => e.join(":")).join(",");
		let i = this.propsOps.get(t);
		if (i === undefined) {
			i = this.propsList.length;
			this.propsOps.set(t, i);
			this.propsList.push(kv);
		}
		return i;
	}
	/** An IRelativePosition {id?, before?, offset?}: its row in the relpos table (streams.py _relpos). */
	relposOf(rp) {
		const marker = rp.id ? this.values.intern(JSON.stringify(rp.id)) : FMT_MT_NO_MARKER;
		this.keys.intern(MARKER_ID_KEY);
		this.relpos.push([marker, rp.offset !== undefined && rp.offset !== null ? rp.offset : 0, rp.before ? FMT_MT_REL_BEFORE : 0]);
		return this.relpos.length - 1;
	}
	/** [pos1, pos2, flags]: getValidOpRange (client.ts:758-767) takes the numbers and falls back to
	 * relativePos1/2 only when they are undefined. */
	positions(op, withPos2) {
		let p1 = op.pos1, p2 = withPos2 ? op.pos2 : undefined, f = 0;
		if ((p1 === undefined || p1 === null) && op.relativePos1 !== undefined && op.relativePos1 !== null) {
			p1 = this.relposOf(op.relativePos1);
			f |= FMT_MT_F_REL1;
		}
		if (withPos2 && (p2 === undefined || p2 === null) && op.relativePos2 !== undefined && op.relativePos2 !== null) {
			p2 = this.relposOf(op.relativePos2);
			f |= FMT_MT_F_REL2;
		}
		return [p1, p2, f];
	}
	/** One raw fmt_mt_op record (the local client's rollback / reconnect records). */
	rawOp(seq, ref, msn, pos1, pos2, payload, len, client, type, flags) {
		const o = this.ops.next();
		const v = this.ops.view;
		v.setInt32(o + 0, seq, true);
		v.setInt32(o + 4, ref, true);
		v.setInt32(o + 8, msn, true);
		v.setInt32(o + 12, pos1, true);
		v.setInt32(o + 16, pos2, true);
		v.setUint32(o + 20, payload, true);
		v.setUint16(o + 24, len, true);
		v.setUint8(o + 26, client);
		v.setUint8(o + 27, type);
		v.setUint32(o + 28, flags, true);
	}
	packOp(op, seq, ref, msn, client, flags) {
		const o = this.ops.next();
		const v = this.ops.view;
		let pos1 = 0, pos2 = 0, payload = 0, len = 0, type = MT_REMOVE;
		if (op !== null) {
			type = op.type;
			if (type === MT_INSERT) {
				const rp = this.positions(op, false);
				flags |= rp[2];
				let seg = op.seg;
				let props = null;
				const rtype = markerRefType(seg);
				if (rtype !== null) { // Marker.make(refType, props): len 1, its arena unit = refType
					const p = seg.props === undefined ? null : seg.props;
					pos1 = rp[0]; pos2 = p === null ? -1 : this.propsOp(p) + 1;
					payload = this.text.push(String.fromCharCode(rtype))[0]; len = 1; flags |= FMT_MT_F_MARKER;
				} else {
					if (typeof seg !== "string") { // IJSONTextSegment {text, props} (textSegment.ts:44-52)
						if (seg && typeof seg === "object" && "text" in seg && Object.keys(seg).every((k) => k === "text" || k === "props")) {
							props = seg.props === undefined ? null : seg.props;
							seg = seg.text;
						} else {
							throw new UnsupportedOp("segment spec");
						}
					}
					const r = this.text.push(seg);
					if (r[1] > 0xffffff) throw new UnsupportedOp("insert longer than 2^24 - 1 UTF-16 units");
					// pos2: the segment's props-op id + 1 (TextSegment.make(text, props)); -1: a plain string
					pos1 = rp[0]; pos2 = props === null ? -1 : this.propsOp(props) + 1; payload = r[0]; len = r[1] & 0xffff;
					flags |= r[1] & FMT_MT_F_LEN_HI_MASK; // length bits 16..23 (fmt.h FMT_MT_F_LEN_HI_SHIFT)
				}
			} else if (type === MT_REMOVE) {
				const rp = this.positions(op, true);
				pos1 = rp[0]; pos2 = rp[1]; flags |= rp[2];
			} else if (type === MT_OBLITERATE) {
				pos1 = op.pos1; pos2 = op.pos2; // non-sided obliterate: {pos1, Before} .. {pos2 - 1, After}
			} else if (type === MT_OBLITERATE_SIDED) {
				pos1 = op.pos1.pos; pos2 = op.pos2.pos;
				flags |= (op.pos1.before ? FMT_MT_F_START_BEFORE : 0) | (op.pos2.before ? FMT_MT_F_END_BEFORE : 0);
			} else if (type === MT_ANNOTATE) { // props (IMergeTreeAnnotateMsg) and/or adjust (IMergeTreeAnnotateAdjustMsg)
				const rp = this.positions(op, true);
				pos1 = rp[0]; pos2 = rp[1]; flags |= rp[2];
				payload = this.propsOp(op.props || {}, op.adjust);
			} else {
				throw new UnsupportedOp(`merge-tree op type ${type}`);
			}
		}
		v.setInt32(o + 0, seq, true);
		v.setInt32(o + 4, ref, true);
		v.setInt32(o + 8, msn, true);
		v.setInt32(o + 12, pos1, true);
		v.setInt32(o + 16, pos2, true);
		v.setUint32(o + 20, payload, true);
		v.setUint16(o + 24, len, true);
		v.setUint8(o + 26, client);
		v.setUint8(o + 27, type);
		v.setUint32(o + 28, flags, true);
	}
	/**
	 * The packed batch: the typed arrays the addon hands to fmt_mt_load. With {catchup: true} the
	 * ops of messages a legacy summary keeps with regenerated contents get FMT_MT_F_CATCHUP: seq
	 * above the document's final minSeq and refSeq != seq - 1 (sequence.ts:949-1018). With
	 * {removeOrder: true} the REMOVE and obliterate ops above the final minSeq (and, in documents
	 * holding obliterates, the INSERTs: obliterate-on-insert) get FMT_MT_F_RMORDER, which the
	 * SnapshotV1 summary needs (summarizeV1).
	 */
	finish(options) {
		const offs = new BigUint64Array(this.docs.length + 1);
		let i = 0;
		this.docs.forEach((d, k) => {
			i += d.nOps;
			offs[k + 1] = BigInt(i);
		});
		if (options && options.removeOrder) {
			const v = this.ops.view;
			let a = 0;
			for (const d of this.docs) {
				const b = a + d.nOps;
				if (b > a) {
					const finalMsn = v.getInt32((b - 1) * MT_OP_BYTES + 8, true);
					const isOb = (t) => t === MT_OBLITERATE || t === MT_OBLITERATE_SIDED;
					let anyOb = false;
					for (let o = a * MT_OP_BYTES; o < b * MT_OP_BYTES; o += MT_OP_BYTES) anyOb = anyOb || isOb(v.getUint8(o + 27));
					for (let o = a * MT_OP_BYTES; o < b * MT_OP_BYTES; o += MT_OP_BYTES) {
						const t = v.getUint8(o + 27);
						if ((v.getUint32(o + 28, true) & FMT_MT_F_LOADSEG) === 0 && v.getInt32(o, true) > finalMsn &&
							(t === MT_REMOVE || isOb(t) || (anyOb && t === MT_INSERT)))
							v.setUint32(o + 28, v.getUint32(o + 28, true) | FMT_MT_F_RMORDER, true);
					}
				}
				a = b;
			}
		}
		if (options && options.catchup) {
			const v = this.ops.view;
			let a = 0;
			for (const d of this.docs) {
				const b = a + d.nOps;
				if (b > a) {
					const finalMsn = v.getInt32((b - 1) * MT_OP_BYTES + 8, true);
					for (let o = a * MT_OP_BYTES; o < b * MT_OP_BYTES; o += MT_OP_BYTES) {
						const seq = v.getInt32(o, true), ref = v.getInt32(o + 4, true);
						if (seq > finalMsn && ref !== seq - 1) v.setUint32(o + 28, v.getUint32(o + 28, true) | FMT_MT_F_CATCHUP, true);
					}
				}
				a = b;
			}
		}
		// value ids: batch-global while the distinct values fit below the id limit, else document-local
		// (fmt.h doc_value_base; streams.py _localize_values)
		const limit = this.adjusts.length ? FMT_MT_VALUE_COMPUTED : FMT_MT_VALUE_ADJUST;
		let propsList = this.propsList, values = this.values.items.slice(), valueBase;
		if (this.values.items.length > limit) [propsList, values, valueBase] = this.localizeValues(limit);
		const propsOff = new Uint32Array(propsList.length + 1);
		const kv = [];
		propsList.forEach((t, j) => {
			for (const e of t) {
				if (e.length === 2) kv.push(((e[0] << 16) | e[1]) >>> 0);
				else kv.push(((e[0] << 16) | FMT_MT_VALUE_ADJUST) >>> 0, e[2]);
			}
			propsOff[j + 1] = kv.length;
		});
		const docInit = new Uint32Array(this.docs.length * 2);
		this.docInit.forEach((p, k) => {
			docInit[2 * k] = p[0];
			docInit[2 * k + 1] = p[1];
		});
		let snapshots, snapshotSegs;
		if (this.snapshots.some((x) => x !== null)) {
			snapshots = new ArrayBuffer(this.docs.length * SNAPSHOT_DOC_BYTES);
			const sv = new DataView(snapshots);
			this.snapshots.forEach((x, k) => {
				if (x === null) return;
				const o = k * SNAPSHOT_DOC_BYTES;
				sv.setBigUint64(o, BigInt(x[0]), true);
				sv.setUint32(o + 8, x[1], true);
				sv.setUint32(o + 12, x[2], true);
				sv.setInt32(o + 16, x[3], true);
				sv.setInt32(o + 20, x[4], true);
				sv.setUint32(o + 24, 1, true);
			});
			snapshotSegs = Uint32Array.from([].concat(...this.snapshotSegs));
		}
		return {
			ops: this.ops.bytes(),
			docOpOffsets: offs,
			snapshots,
			snapshotSegs,
			text: this.text.finish(),
			docInit,
			propsOff,
			propsKv: Uint32Array.from(kv),
			keys: this.keys.items.slice(),
			values,
			docValueBase: valueBase,
			clients: this.docs.map((d) => d.clientNames.slice()),
			messages: this.docs.map((d) => d.messages),
			nDocs: this.docs.length,
			relpos: this.relpos.length ? Uint32Array.from([].concat(...this.relpos.map((r) => [r[0], r[1] >>> 0, r[2], 0]))) : undefined,
			snapshotInfo: this.hasMergeInfo ? Uint32Array.from([].concat(...this.snapshotInfo.map((r) => [r[0] >>> 0, r[1] >>> 0, r[2], r[3]]))) : undefined,
			snapshotStamps: this.hasMergeInfo ? Uint32Array.from([].concat(...this.snapshotStamps.map((r) => [r[0] >>> 0, r[1] >>> 0, r[2], 0]))) : undefined,
			markerIdKey: this.relpos.length && this.keys.ids.has(MARKER_ID_KEY) ? this.keys.ids.get(MARKER_ID_KEY) : FMT_MT_NO_MARKER,
			adjusts: this.adjusts.length ? adjustBytes(this.adjusts) : undefined,
			valueNum: this.adjusts.length ? Float64Array.from(values, valueNumber) : undefined,
		};
	}
	/**
	 * Document-local value ids: every props op a document references (annotate payloads, insert props
	 * pos2 - 1, its summary segments' props) becomes a props op of that document alone whose values
	 * are numbered 1.. in the document's own dictionary; its relative positions' marker ids follow.
	 * Rewrites the op records and segment / relpos rows in place. Mirrors streams.py _localize_values.
	 */
	localizeValues(limit) {
		const v = this.ops.view;
		const pairs = new Map(); // "doc:pid" -> new props op id
		const list = [];
		const local = this.docs.map(() => new Map()); // per document: batch value id -> local id
		const lid = (d, g) => {
			const m = local[d];
			let x = m.get(g);
			if (x === undefined) {
				x = m.size + 1;
				m.set(g, x);
			}
			return x;
		};
		const refs = []; // [doc, pid, apply(newPid)]
		let a = 0;
		this.docs.forEach((doc, d) => {
			for (let i = a; i < a + doc.nOps; i++) {
				const o = i * MT_OP_BYTES, t = v.getUint8(o + 27);
				if (t === MT_ANNOTATE) refs.push([d, v.getUint32(o + 20, true), (p) => v.setUint32(o + 20, p, true)]);
				else if (t === MT_INSERT && v.getInt32(o + 16, true) > 0)
					refs.push([d, v.getInt32(o + 16, true) - 1, (p) => v.setInt32(o + 16, p + 1, true)]);
			}
			a += doc.nOps;
		});
		this.snapshotSegs.forEach((sg, k) => {
			if (sg[2] !== NO_PROPS) refs.push([this.segDoc[k], sg[2], (p) => { sg[2] = p; }]);
		});
		refs.sort((x, y) => x[0] - y[0] || x[1] - y[1]);
		for (const [d, pid, apply] of refs) {
			const key = `${d}:${pid}`;
			let np = pairs.get(key);
			if (np === undefined) {
				np = list.length;
				pairs.set(key, np);
				list.push(this.propsList[pid].map((e) => (e.length === 2 ? [e[0], e[1] === 0 ? 0 : lid(d, e[1])] : e)));
			}
			apply(np);
		}
		a = 0;
		this.docs.forEach((doc, d) => {
			for (let i = a; i < a + doc.nOps; i++) {
				const o = i * MT_OP_BYTES, f = v.getUint32(o + 28, true);
				for (const [flag, at] of [[FMT_MT_F_REL1, 12], [FMT_MT_F_REL2, 16]]) {
					if ((f & flag) === 0) continue;
					const row = this.relpos[v.getInt32(o + at, true)];
					if (row[0] !== FMT_MT_NO_MARKER) row[0] = lid(d, row[0]);
				}
			}
			a += doc.nOps;
		});
		const values = ["null"], base = new Uint32Array(this.docs.length + 1);
		local.forEach((m, d) => {
			if (m.size >= limit) throw new UnsupportedOp(`more than ${limit - 1} distinct property values in one document`);
			base[d] = values.length - 1;
			for (const g of m.keys()) values.push(this.values.items[g]);
		});
		base[this.docs.length] = values.length - 1;
		return [list, values, base];
	}
}

/** Document d's value table (value id -> JSON text): the batch's, or its own slice when the batch
 * has document-local value ids (docValueBase, fmt.h doc_value_base). */
function docValues(batch, d) {
	if (!batch.docValueBase) return batch.values;
	return ["null"].concat(batch.values.slice(batch.docValueBase[d] + 1, batch.docValueBase[d + 1] + 1));
}

/** fmt_mt_adjust rows (32 bytes: f64 delta, min, max, u32 flags, pad) as bytes. */
function adjustBytes(rows) {
	const b = new ArrayBuffer(32 * rows.length);
	const v = new DataView(b);
	rows.forEach((r, i) => {
		v.setFloat64(32 * i, r[0], true);
		v.setFloat64(32 * i + 8, r[1], true);
		v.setFloat64(32 * i + 16, r[2], true);
		v.setUint32(32 * i + 24, r[3], true);
	});
	return new Uint8Array(b);
}

/** The number a value's JSON text holds (typeof "number" after JSON.parse), else NaN. */
function valueNumber(text) {
	try {
		const v = JSON.parse(text);
		return typeof v === "number" ? v : NaN;
	} catch (e) {
		return NaN;
	}
}

/** Packs SharedMap messages (mirror of streams.py MapStreamBuilder; mapKernel.ts:706-853 kinds). */
class MapStreamBuilder {
	constructor() {
		this.keys = new Dictionary();
		this.values = new Dictionary();
		this.ops = new RecordBuffer(MAP_OP_BYTES);
		this.docOps = [];
		this.events = new RecordBuffer(MAP_OP_BYTES);  // fmt_map_local_op records (same 16-byte shape)
		this.docEvents = [];
		this.unacked = [];
	}
	beginDoc() {
		this.docOps.push(0);
		this.docEvents.push(0);
		this.unacked = [];
		this.lastSeq = 0;
		return this.docOps.length - 1;
	}
	/** (key id, kind_value) of a set / delete / clear op's contents. */
	record(contents) {
		if (contents.type === "clear") return [0, (MAP_CLEAR << MAP_KIND_SHIFT) >>> 0];
		if (contents.type !== "set" && contents.type !== "delete") throw new UnsupportedOp(`map op type ${contents.type}`);
		const key = this.keys.intern(contents.key);
		if (contents.type === "delete") return [key, (MAP_DELETE << MAP_KIND_SHIFT) >>> 0];
		const sv = contents.value;
		if (sv.type !== "Plain") throw new UnsupportedOp("legacy Shared value type");
		let vid = MAP_VALUE_UNDEFINED;
		if ("value" in sv && sv.value !== undefined) {
			vid = this.values.intern(JSON.stringify(sv.value));
			if (vid >= MAP_VALUE_UNDEFINED) throw new UnsupportedOp("value dictionary overflow");
		}
		return [key, ((MAP_SET << MAP_KIND_SHIFT) | vid) >>> 0];
	}
	pushEvent(doc, key, event, kv) {
		const o = this.events.next();
		const v = this.events.view;
		v.setUint32(o, doc, true);
		v.setUint32(o + 4, key, true);
		v.setUint32(o + 8, event, true);
		v.setUint32(o + 12, kv, true);
		this.docEvents[doc]++;
	}
	/**
	 * The document's local client (MapKernel pendingData, mapKernel.ts:132-139): set / delete / clear
	 * on the attached map enters pendingData (:388-538) until its ack; rollback drops the newest
	 * (:633-700).
	 */
	localSubmit(doc, contents) {
		if (doc !== this.docOps.length - 1) throw new UnsupportedOp("documents must be packed contiguously");
		const [key, kv] = this.record(contents);
		this.pushEvent(doc, key, MAP_EV_SUBMIT, kv);
		this.unacked.push([key, kv]);
	}
	/** The oldest pending local op comes back sequenced (the handlers' local branches, :706-853). */
	localAck(doc, seq) {
		if (this.unacked.length === 0) throw new Error("localAck with no unacknowledged local op");
		if (seq < this.lastSeq) throw new Error(`map message seq ${seq} after ${this.lastSeq}: messages must arrive in seq order`);
		this.lastSeq = seq;
		const [key, kv] = this.unacked.shift();
		const o = this.ops.next();
		const v = this.ops.view;
		v.setUint32(o, doc, true);
		v.setUint32(o + 4, key, true);
		v.setUint32(o + 8, this.docOps[doc] + 1, true);
		v.setUint32(o + 12, kv, true);
		this.docOps[doc]++;
		this.pushEvent(doc, key, MAP_EV_ACK, kv);
	}
	localRollback(doc) {
		if (this.unacked.length === 0) throw new Error("localRollback with no unacknowledged local op");
		const [key, kv] = this.unacked.pop();
		this.pushEvent(doc, key, MAP_EV_ROLLBACK, kv);
	}
	/**
	 * One sequenced map message. Messages of one bunch share their envelope's sequenceNumber
	 * (sharedObject.ts:620-630), so the record carries the message's 1-based ordinal in the document
	 * instead: strictly increasing, it keeps a bunch's order for LWW and JS Map insertion order.
	 */
	addMessage(doc, seq, contents) {
		if (doc !== this.docOps.length - 1) throw new UnsupportedOp("documents must be packed contiguously");
		if (seq < this.lastSeq) throw new Error(`map message seq ${seq} after ${this.lastSeq}: messages must arrive in seq order`);
		this.lastSeq = seq;
		const ordinal = this.docOps[doc] + 1;
		const o = this.ops.next();
		const v = this.ops.view;
		let key = 0, kv;
		if (contents.type === "clear") {
			kv = (MAP_CLEAR << MAP_KIND_SHIFT) >>> 0;
		} else if (contents.type === "delete") {
			key = this.keys.intern(contents.key);
			kv = (MAP_DELETE << MAP_KIND_SHIFT) >>> 0;
		} else if (contents.type === "set") {
			key = this.keys.intern(contents.key);
			const sv = contents.value;
			if (sv.type !== "Plain") throw new UnsupportedOp("legacy Shared value type");
			let vid = MAP_VALUE_UNDEFINED;
			if ("value" in sv && sv.value !== undefined) {
				vid = this.values.intern(JSON.stringify(sv.value));
				if (vid >= MAP_VALUE_UNDEFINED) throw new UnsupportedOp("value dictionary overflow");
			}
			kv = ((MAP_SET << MAP_KIND_SHIFT) | vid) >>> 0;
		} else {
			throw new UnsupportedOp(`map op type ${contents.type}`);
		}
		v.setUint32(o, doc, true);
		v.setUint32(o + 4, key, true);
		v.setUint32(o + 8, ordinal, true);
		v.setUint32(o + 12, kv, true);
		this.docOps[doc]++;
	}
	/**
	 * A document whose map starts from a SharedMap summary (SharedMap.loadCore, map.ts:251-267): the
	 * header's "content" entries, then each blob's, in Object.entries order
	 * (populateFromSerializable, mapKernel.ts:557-564), packed as the document's first set records.
	 */
	beginDocFromSummary(header, blobs) {
		const doc = this.beginDoc();
		const h = JSON.parse(header);
		const parts = Array.isArray(h.blobs) ? [h.content].concat((blobs || []).map((b) => JSON.parse(b))) : [h];
		for (const part of parts) {
			for (const [key, ser] of Object.entries(part)) {
				const value = { type: ser.type === undefined ? "Plain" : ser.type };
				if ("value" in ser) value.value = ser.value;
				this.addMessage(doc, 0, { type: "set", key, value });
			}
		}
		return doc;
	}
	/** SharedMap.processMessagesCore shape (map.ts:288-311): one bunch for document `doc`. */
	processMessagesCore(doc, messagesCollection) {
		for (const mc of messagesCollection.messagesContent) {
			this.addMessage(doc, messagesCollection.envelope.sequenceNumber, mc.contents);
		}
	}
	finish() {
		const offs = new BigUint64Array(this.docOps.length + 1);
		let i = 0;
		this.docOps.forEach((n, k) => {
			i += n;
			offs[k + 1] = BigInt(i);
		});
		const out = {
			ops: this.ops.bytes(),
			docOpOffsets: offs,
			keyBound: Math.max(1, this.keys.items.length),
			keys: this.keys.items.slice(),
			values: this.values.items.slice(),
			nDocs: this.docOps.length,
		};
		if (this.docEvents.some((n) => n > 0)) {
			const eo = new BigUint64Array(this.docEvents.length + 1);
			let e = 0;
			this.docEvents.forEach((n, k) => {
				e += n;
				eo[k + 1] = BigInt(e);
			});
			out.localOps = this.events.bytes();
			out.localOffsets = eo;
		}
		return out;
	}
}

function readHeader(dv, d) {
	const o = d * DOC_RESULT_BYTES;
	return {
		status: dv.getInt32(o, true),
		failSeq: dv.getInt32(o + 4, true),
		curSeq: dv.getInt32(o + 8, true),
		minSeq: dv.getInt32(o + 12, true),
		nLeaves: dv.getUint32(o + 16, true),
		nChars: dv.getUint32(o + 20, true),
		nProps: dv.getUint32(o + 24, true),
		nBlocks: dv.getUint32(o + 28, true),
		depth: dv.getUint32(o + 32, true),
		visibleLength: dv.getUint32(o + 36, true),
		nCatchup: dv.getUint32(o + 40, true),
		nRmOrder: dv.getUint32(o + 44, true),
	};
}

/** Converged state of a replayed merge-tree batch (read side of SharedString). */
class MergeTreeReplay {
	constructor(engine, batch, headers) {
		this.engine = engine;
		this.batch = batch;
		this.headerView = new DataView(headers);
	}
	header(doc) {
		return readHeader(this.headerView, doc);
	}
	/** The document's computed annotate-adjust numbers (value ids FMT_MT_VALUE_COMPUTED + k). */
	numbers(doc) {
		return this.batch.adjusts ? native().fetchNumbers(this.engine.ctx, doc) : new Float64Array(0);
	}
	/** The value texts the document's prop sets index: the batch's, then its computed numbers. */
	valuesOf(doc) {
		const nums = this.numbers(doc);
		const own = docValues(this.batch, doc);
		if (nums.length === 0) return own;
		const vals = own.slice();
		nums.forEach((x, k) => { vals[FMT_MT_VALUE_COMPUTED + k] = JSON.stringify(x); });
		return vals;
	}
	/** Leaves (segments, tombstones included), UTF-16 chars and prop sets of one document. */
	segments(doc) {
		const h = this.header(doc);
		if (h.status !== 0) {
			const e = new Error(`document ${doc} failed at seq ${h.failSeq} (status ${h.status})`);
			e.code = h.status === -2 ? "FMT_E_DATA" : h.status === -3 ? "FMT_E_CAPACITY" : "FMT_E_UNSUPPORTED";
			throw e;
		}
		const r = native().fetchDoc(this.engine.ctx, doc, h.nLeaves, h.nChars, h.nProps);
		const lv = new DataView(r.leaves), pv = new DataView(r.props);
		const chars = new Uint16Array(r.chars);
		const nums = this.numbers(doc);
		const vals = docValues(this.batch, doc);
		// entry k of the set whose first record is p (a set wider than PROPS_MAX continues in the next
		// records, fmt.h fmt_mt_propset; continuation records have n = FMT_MT_PROPS_CONT)
		const entry = (p, k) => pv.getUint32((p + Math.floor(k / PROPS_MAX)) * PROPSET_BYTES + 4 + 4 * (k % PROPS_MAX), true);
		const width = (p) => {
			const n = pv.getUint32(p * PROPSET_BYTES, true);
			return n === FMT_MT_PROPS_CONT || p + Math.floor((n - 1) / PROPS_MAX) >= h.nProps ? 0 : n;
		};
		const props = [];
		for (let p = 0; p < h.nProps; p++) {
			const n = width(p);
			const obj = {};
			for (let k = 0; k < n; k++) {
				const kv = entry(p, k);
				const val = kv & 0xffff;
				if (val !== 0) {
					obj[this.batch.keys[kv >>> 16]] = val >= FMT_MT_VALUE_COMPUTED && this.batch.adjusts
						? nums[val - FMT_MT_VALUE_COMPUTED] : JSON.parse(vals[val]);
				}
			}
			props.push(obj);
		}
		const kvs = [];
		for (let p = 0; p < h.nProps; p++) {
			const n = width(p);
			const kv = [];
			for (let k = 0; k < n; k++) kv.push(entry(p, k));
			kvs.push(kv);
		}
		const segs = [];
		segs.kvs = kvs; // every prop set's (key, value) ids, by set id
		for (let i = 0; i < h.nLeaves; i++) {
			const o = i * LEAF_BYTES;
			const off = lv.getUint32(o + 16, true), len = lv.getUint32(o + 20, true);
			const pid = lv.getUint16(o + 26, true);
			const rm = lv.getInt32(o + 4, true);
			const marker = (lv.getUint16(o + 30, true) & FMT_MT_LEAF_MARKER) !== 0;
			segs.push({
				marker, // a Marker segment: its one char unit is its refType
				refType: marker ? chars[off] : undefined,
				insertSeq: lv.getInt32(o, true),
				removedSeq: rm === NOT_REMOVED ? undefined : rm,
				insertClient: lv.getInt16(o + 24, true),
				text: String.fromCharCode.apply(null, chars.subarray(off, off + len)),
				properties: pid === 0xffff ? undefined : props[pid],
				kv: pid === 0xffff ? null : kvs[pid],
			});
		}
		return segs;
	}
	/** Props op `id` of the batch as the object it was packed from (null values: deletions). */
	propsOf(doc, id) {
		const vals = docValues(this.batch, doc);
		const out = {};
		for (let t = this.batch.propsOff[id]; t < this.batch.propsOff[id + 1]; t++) {
			const kv = this.batch.propsKv[t], val = kv & 0xffff;
			out[this.batch.keys[kv >>> 16]] = val === 0 ? null : JSON.parse(vals[val]);
		}
		return out;
	}
	/**
	 * f4: what regeneratePendingOp returned at each reconnect record of the document
	 * (client.ts:1452-1542, one op per segment of each pending op, in order), as
	 * [{localSeq, refSeq, op}] with op an IMergeTreeInsertMsg / RemoveMsg / AnnotateMsg in the
	 * reconnect view — the ops to resubmit (fmt_mt_fetch_regen).
	 */
	regenerated(doc) {
		const r = native().fetchRegen(this.engine.ctx, doc);
		const dv = new DataView(r.ops);
		const out = [];
		for (let o = 0; o < r.ops.byteLength; o += MT_OP_BYTES) {
			const type = dv.getUint8(o + 27), flags = dv.getUint32(o + 28, true);
			const pos1 = dv.getInt32(o + 12, true), pos2 = dv.getInt32(o + 16, true), payload = dv.getUint32(o + 20, true);
			let op;
			if (type === MT_INSERT) {
				const n = dv.getUint16(o + 24, true) + (flags & FMT_MT_F_LEN_HI_MASK);
				const props = pos2 > 0 ? this.propsOf(doc, pos2 - 1) : undefined;
				let seg;
				if (flags & FMT_MT_F_MARKER) {
					seg = { marker: { refType: r.text[payload] } };
					if (props) seg.props = props;
				} else {
					const text = String.fromCharCode.apply(null, r.text.subarray(payload, payload + n));
					seg = props ? { text, props } : text;
				}
				op = { type, pos1, seg };
			} else if (type === MT_REMOVE) {
				op = { type, pos1, pos2 };
			} else {
				op = { type, pos1, pos2, props: this.propsOf(doc, payload) };
			}
			out.push({ localSeq: dv.getInt32(o, true), refSeq: dv.getInt32(o + 4, true), op });
		}
		return out;
	}
	/** The document's catch-up ranges (ops flagged by finish({catchup: true})). */
	catchupRanges(doc) {
		const n = this.header(doc).nCatchup;
		const dv = new DataView(native().fetchCatchup(this.engine.ctx, doc, n));
		const out = [];
		for (let i = 0; i < n; i++) {
			const o = i * CATCHUP_BYTES;
			out.push({ op: dv.getUint32(o, true), pos1: dv.getInt32(o + 4, true), pos2: dv.getInt32(o + 8, true),
				type: dv.getUint32(o + 12, true) });
		}
		return out;
	}
	/**
	 * SharedString.summarizeCore legacy blobs at the document's minSeq (snapshotlegacy.ts:126-262):
	 * {header, body (or undefined), catchupOps (or undefined)}. catchupOps needs a batch built with
	 * keepMessages and finish({catchup: true}).
	 */
	summarize(doc) {
		const h = this.header(doc);
		const all = this.segments(doc);
		// getAtSeq(properties, minSeq) (snapshotlegacy.ts:211-212): with annotate-adjust the engine's
		// per-leaf prop sets of each segment's PropertiesManager at minSeq
		const legacy = this.batch.adjusts ? native().fetchLegacyProps(this.engine.ctx, doc, h.nLeaves) : null;
		const segs = all.map((s, i) => ({
			insertSeq: s.insertSeq,
			removedSeq: s.removedSeq === undefined ? NOT_REMOVED : s.removedSeq,
			text: s.text,
			kv: legacy ? (legacy[i] === 0xffff ? null : all.kvs[legacy[i]]) : s.kv,
			refType: s.refType,
		}));
		const out = summary.legacySummary(segs, h.minSeq, this.batch.keys, this.valuesOf(doc));
		const msgs = this.batch.messages && this.batch.messages[doc];
		if (msgs && msgs.length) {
			const cu = summary.catchupMessages(msgs, this.catchupRanges(doc), h.minSeq);
			if (cu.length) out.catchupOps = JSON.stringify(cu);
		}
		return out;
	}
	/**
	 * The remove stamps of every removed leaf in stamp order: the first is the op whose seq is the
	 * leaf's removedSeq (its client; kind 0 for a REMOVE, 1 for an obliterate), later ones come from
	 * the kernel's remove-order slab (ops flagged by finish({removeOrder: true})), sorted by seq.
	 * {leaf index: [[short client id, seq, kind], ...]}.
	 */
	removers(doc, segs) {
		const h = this.header(doc);
		const first = new Map();
		const ops = new DataView(this.batch.ops.buffer, this.batch.ops.byteOffset, this.batch.ops.byteLength);
		for (let i = Number(this.batch.docOpOffsets[doc]); i < Number(this.batch.docOpOffsets[doc + 1]); i++) {
			const seq = ops.getInt32(i * MT_OP_BYTES, true), t = ops.getUint8(i * MT_OP_BYTES + 27);
			if ((t === MT_REMOVE || t === MT_OBLITERATE || t === MT_OBLITERATE_SIDED) && !first.has(seq))
				first.set(seq, [ops.getUint8(i * MT_OP_BYTES + 26), t === MT_REMOVE ? 0 : 1]);
		}
		const out = {};
		segs.forEach((s, i) => {
			if (s.removedSeq !== undefined && first.has(s.removedSeq)) {
				const f = first.get(s.removedSeq);
				out[i] = [[f[0], s.removedSeq, f[1]]];
			}
		});
		const later = {};
		const dv = new DataView(native().fetchRemoveOrder(this.engine.ctx, doc, h.nRmOrder));
		for (let k = 0; k < h.nRmOrder; k++) { // fmt_mt_remove_order: leaf, client, seq, kind (16 B)
			const leaf = dv.getUint32(16 * k, true);
			if (leaf !== 0xffffffff && out[leaf])
				(later[leaf] = later[leaf] || []).push([dv.getInt32(16 * k + 4, true), dv.getInt32(16 * k + 8, true),
					dv.getUint32(16 * k + 12, true)]);
		}
		for (const leaf of Object.keys(later)) {
			const es = later[leaf].map((e, k) => [e, k]).sort((x, y) => x[0][1] - y[0][1] || x[1] - y[1]);
			for (const e of es) out[leaf].push(e[0]);
		}
		return out;
	}
	/**
	 * SharedString.summarizeCore in the SnapshotV1 format (newMergeTreeSnapshotFormat,
	 * snapshotV1.ts:90-265): {header, bodies} for the blobs header, body_0, body_1, ...
	 */
	summarizeV1(doc) {
		const h = this.header(doc);
		const segs = this.segments(doc);
		const rem = this.removers(doc, segs);
		const v1 = segs.map((s) => ({
			insertSeq: s.insertSeq,
			insertClient: s.insertClient,
			removedSeq: s.removedSeq === undefined ? NOT_REMOVED : s.removedSeq,
			text: s.text,
			kv: s.kv,
			refType: s.refType,
		}));
		return summary.v1Summary(v1, h.minSeq, h.curSeq, this.batch.keys, this.valuesOf(doc), this.batch.clients[doc], rem);
	}
	/**
	 * Legacy summaries of every document at once on the device (fmt_mt_summarize_legacy: the
	 * extractSync merge in one launch, JSON on host threads). Resolves to the timing; read each
	 * document's blobs with legacyBlobs(doc). Catch-up ops are not part of this path (summarize(doc)
	 * builds them).
	 */
	async summarizeAllLegacy(options) {
		const o = options || {};
		const t = await native().summarizeLegacy(this.engine.ctx, this.batch.keys.map((k) => JSON.stringify(k)), this.batch.values,
			o.chunkSize || 10000, o.threads || 0);
		// the catchupOps blobs (snapshotlegacy.ts:178-190): every document's catch-up ranges in one copy
		// (fmt_mt_fetch_catchup_all), messages rebuilt here from the kept messages
		this.bulkCatchup = null;
		if (this.batch.messages && this.batch.messages.some((m) => m && m.length)) {
			const t0 = Date.now();
			const all = native().fetchCatchupAll(this.engine.ctx, this.batch.nDocs);
			this.bulkCatchup = { offsets: all.offsets, dv: new DataView(all.ranges) };
			t.catchupFetchMs = Date.now() - t0;
		}
		return t;
	}
	/**
	 * {header, body?, catchupOps?} of document doc from the last summarizeAllLegacy (throws with its
	 * status). catchupOps needs a batch built with keepMessages and finish({catchup: true}).
	 */
	legacyBlobs(doc) {
		const out = native().summaryBlobs(this.engine.ctx, doc);
		const msgs = this.batch.messages && this.batch.messages[doc];
		if (this.bulkCatchup && msgs && msgs.length) {
			const { offsets, dv } = this.bulkCatchup;
			const ranges = [];
			for (let i = offsets[doc]; i < offsets[doc + 1]; i++) {
				const o = i * CATCHUP_BYTES;
				ranges.push({ op: dv.getUint32(o, true), pos1: dv.getInt32(o + 4, true), pos2: dv.getInt32(o + 8, true),
					type: dv.getUint32(o + 12, true) });
			}
			const cu = summary.catchupMessages(msgs, ranges, this.header(doc).minSeq);
			if (cu.length) out.catchupOps = JSON.stringify(cu);
		}
		return out;
	}
	/** MergeTreeTextHelper.getText from the local perspective (MergeTreeTextHelper.ts:28-87). */
	getText(doc) {
		return this.segments(doc).filter((s) => s.removedSeq === undefined && !s.marker).map((s) => s.text).join("");
	}
	getLength(doc) {
		return this.header(doc).visibleLength;
	}
}

/** Converged SharedMap state (MapKernel.sequencedData, mapKernel.ts:131). */
class MapReplay {
	constructor(batch, slots) {
		this.batch = batch;
		this.view = new DataView(slots);
	}
	/** Live entries in JS Map iteration order (insertion = birth seq of the live entry). */
	entries(doc) {
		const kb = this.batch.keyBound;
		const live = [];
		for (let k = 0; k < kb; k++) {
			const o = (doc * kb + k) * 8;
			const value = this.view.getUint32(o, true);
			if (value === MAP_ABSENT) continue;
			live.push([this.view.getUint32(o + 4, true), k, value]);
		}
		live.sort((a, b) => a[0] - b[0] || a[1] - b[1]);
		return live.map(([, k, v]) => [this.batch.keys[k],
			v === MAP_VALUE_UNDEFINED ? undefined : JSON.parse(this.batch.values[v])]);
	}
	/** SharedMap.summarizeCore blobs (map.ts:176-246): {header, blobs}. */
	summarize(doc) {
		const kb = this.batch.keyBound;
		const live = [];
		for (let k = 0; k < kb; k++) {
			const o = (doc * kb + k) * 8;
			const value = this.view.getUint32(o, true);
			if (value !== MAP_ABSENT) live.push([this.view.getUint32(o + 4, true), k, value]);
		}
		live.sort((a, b) => a[0] - b[0] || a[1] - b[1]);
		return summary.mapSummary(live.map(([, k, v]) => [this.batch.keys[k],
			v === MAP_VALUE_UNDEFINED ? undefined : this.batch.values[v]]));
	}
	get(doc, key) {
		const k = this.batch.keys.indexOf(key);
		if (k < 0) return undefined;
		const value = this.view.getUint32((doc * this.batch.keyBound + k) * 8, true);
		if (value === MAP_ABSENT || value === MAP_VALUE_UNDEFINED) return undefined;
		return JSON.parse(this.batch.values[value]);
	}
}

/** Converged SharedMap state from the sparse path (key pools of any size): live entries per
 * document in JS Map insertion order (fmt_map_entry records). */
class SparseMapReplay {
	constructor(batch, counts, entries, pending) {
		this.batch = batch;
		this.counts = new Uint32Array(counts);
		this.view = new DataView(entries);
		this.first = new Float64Array(this.counts.length + 1);
		for (let d = 0; d < this.counts.length; d++) this.first[d + 1] = this.first[d] + this.counts[d];
		if (pending !== undefined) {  // the local client's optimistic view (fmt_map_pending_*)
			this.pCounts = new Uint32Array(pending.counts);
			this.pStatus = new Int32Array(pending.status);
			this.pView = new DataView(pending.entries);
			this.pFirst = new Float64Array(this.pCounts.length + 1);
			for (let d = 0; d < this.pCounts.length; d++) this.pFirst[d + 1] = this.pFirst[d] + this.pCounts[d];
		}
	}
	/**
	 * The local client's view of document doc (MapKernel's internalIterator over sequencedData and
	 * pendingData, mapKernel.ts:176-240): [[key, value], ...] in its iteration order.
	 */
	optimisticEntries(doc) {
		if (this.pCounts === undefined) return this.entries(doc);
		if (this.pStatus[doc] !== 0) {
			const e = new Error(`document ${doc}: local events do not match its pending ops`);
			e.code = "FMT_E_DATA";
			throw e;
		}
		const out = [];
		for (let i = this.pFirst[doc]; i < this.pFirst[doc + 1]; i++) {
			const k = this.pView.getUint32(i * 12, true), v = this.pView.getUint32(i * 12 + 4, true);
			out.push([this.batch.keys[k], v === MAP_VALUE_UNDEFINED ? undefined : JSON.parse(this.batch.values[v])]);
		}
		return out;
	}
	/** MapKernel.get (:374-392): the optimistic value. */
	optimisticGet(doc, key) {
		const e = this.optimisticEntries(doc).find(([k]) => k === key);
		return e === undefined ? undefined : e[1];
	}
	/** [[key id, value id, birth seq], ...] of document doc in birth order. */
	rawEntries(doc) {
		const out = [];
		for (let i = this.first[doc]; i < this.first[doc + 1]; i++) {
			const o = i * 12;
			out.push([this.view.getUint32(o, true), this.view.getUint32(o + 4, true), this.view.getUint32(o + 8, true)]);
		}
		return out;
	}
	entries(doc) {
		return this.rawEntries(doc).map(([k, v]) => [this.batch.keys[k],
			v === MAP_VALUE_UNDEFINED ? undefined : JSON.parse(this.batch.values[v])]);
	}
	summarize(doc) {
		return summary.mapSummary(this.rawEntries(doc).map(([k, v]) => [this.batch.keys[k],
			v === MAP_VALUE_UNDEFINED ? undefined : this.batch.values[v]]));
	}
	get(doc, key) {
		const e = this.rawEntries(doc).find(([k]) => this.batch.keys[k] === key);
		return e === undefined || e[1] === MAP_VALUE_UNDEFINED ? undefined : JSON.parse(this.batch.values[e[1]]);
	}
}

/** One engine context on one GPU (fmt_open). */
class Engine {
	constructor(device) {
		this.ctx = native().open(device === undefined ? 0 : device);
	}
	deviceInfo() {
		return native().deviceInfo(this.ctx);
	}
	stats() {
		return native().stats(this.ctx);
	}
	async replayMergeTree(batch) {
		const headers = await native().replayMergeTree(this.ctx, batch);
		return new MergeTreeReplay(this, batch, headers);
	}
	async replayMap(batch) {
		const slots = await native().replayMap(this.ctx, batch);
		return new MapReplay(batch, slots);
	}
	/** The sparse LWW path (fmt_map_*_sparse): any key pool size, live entries only. */
	async replayMapSparse(batch) {
		const r = await native().replayMapSparse(this.ctx, batch);
		return new SparseMapReplay(batch, r.counts, r.entries, r.pending);
	}
	close() {
		native().close(this.ctx);
	}
}

module.exports = {
	native,
	Engine,
	MergeTreeStreamBuilder,
	MapStreamBuilder,
	MergeTreeReplay,
	MapReplay,
	SparseMapReplay,
	UnsupportedOp,
	summary,
	constants: { MT_INSERT, MT_REMOVE, MT_ANNOTATE, MT_GROUP, MAP_SET, MAP_DELETE, MAP_CLEAR,
		MAP_VALUE_UNDEFINED, MAP_ABSENT, FMT_MT_F_GROUP_CONT, FMT_MT_F_CATCHUP, NOT_REMOVED,
		FMT_MT_F_LOCAL, FMT_MT_F_ACK, FMT_MT_F_ROLLBACK, FMT_MT_F_REGEN, FMT_MT_LOCAL_SEQ_BASE: 0x40000000 },
};
