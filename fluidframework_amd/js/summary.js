"use strict";
/**
 * summary.js — summarizeCore from converged engine state, in JavaScript (the addon's read side).
 *
 * JavaScript twin of fluidframework_amd/summary.py; both emit the bytes the reference's
 * summarizeCore emits:
 *   SharedMap.summarizeCore                 packages/dds/map/src/map.ts:176-246
 *     over MapKernel.getSerializedStorage   map/src/mapKernel.ts:545-551 (Object order of the Map)
 *   SharedString legacy summary             merge-tree/src/snapshotlegacy.ts:74-262 (extractSync, emit)
 *     chunk format                          merge-tree/src/snapshotChunks.ts:85-204
 *     catch-up ops                          sequence/src/sequence.ts:395-452, 949-1018
 * Here JSON.stringify does the serialising, so JS key order comes for free.
 */
const MT_INSERT = 0, MT_REMOVE = 1, MT_GROUP = 3, MT_OBLITERATE = 4;
const NOT_REMOVED = 0x7fffffff;
const TEXT_GRANULARITY = 256; // textSegment.ts:21
const SIZE_OF_FIRST_CHUNK = 10000; // snapshotlegacy.ts:55
const MIN_VALUE_SIZE_SEPARATE_BLOB = 8 * 1024; // map.ts:190
const MAX_SNAPSHOT_BLOB_SIZE = 16 * 1024; // map.ts:194

/**
 * SharedMap summary of one document.
 * @param entries - live [key, valueJsonText | undefined] pairs in Map insertion order.
 * @returns {{header: string, blobs: string[]}} the "header" blob and blob0.. in order.
 */
function mapSummary(entries) {
	const data = {}; // getSerializedStorage: a plain object, so array-index keys enumerate first
	for (const [key, json] of entries) data[key] = { type: "Plain", value: json };
	let currentSize = 0;
	let headerBlob = {};
	const blobs = [];
	const blobTexts = [];
	for (const [key, value] of Object.entries(data)) {
		if (value.value && value.value.length >= MIN_VALUE_SIZE_SEPARATE_BLOB) {
			blobs.push(`blob${blobs.length}`);
			blobTexts.push(JSON.stringify({ [key]: { type: value.type, value: JSON.parse(value.value) } }));
		} else {
			currentSize += value.type.length + 21;
			if (value.value) currentSize += value.value.length;
			if (currentSize > MAX_SNAPSHOT_BLOB_SIZE) {
				blobs.push(`blob${blobs.length}`);
				blobTexts.push(JSON.stringify(headerBlob));
				headerBlob = {};
				currentSize = 0;
			}
			headerBlob[key] = {
				type: value.type,
				value: value.value === undefined ? undefined : JSON.parse(value.value),
			};
		}
	}
	return { header: JSON.stringify({ blobs, content: headerBlob }), blobs: blobTexts };
}

/** properties.ts:32-61 on (key, value) id lists; undefined matches {}. */
function propsMatch(a, b) {
	a = a || [];
	b = b || [];
	if (a.length !== b.length) return false;
	const bk = new Map(b.map((x) => [x >>> 16, x]));
	return a.every((x) => bk.get(x >>> 16) === x);
}

function propsObject(kv, keys, values) {
	const o = {};
	for (const x of kv) o[keys[x >>> 16]] = JSON.parse(values[x & 0xffff]);
	return o;
}

/**
 * extractSync (snapshotlegacy.ts:195-262): segments present at PriorPerspective(minSeq,
 * NonCollabClient), each appended onto the previous while canAppend && matchProperties.
 * @param segs - the document's leaves in order: {insertSeq, removedSeq (or NOT_REMOVED), text, kv}
 *   with kv the prop-set's (key << 16 | value) ids, or null when properties are undefined.
 */
function legacySegments(segs, minSeq) {
	const out = [];
	for (const s of segs) {
		if (!(s.insertSeq <= minSeq) || s.removedSeq <= minSeq) continue;
		const prev = out[out.length - 1];
		// canAppend: both TextSegments (a Marker never appends, mergeTreeNodes.ts:557-559)
		if (prev && prev.refType === undefined && s.refType === undefined && !prev.text.endsWith("\n") &&
			(prev.text.length <= TEXT_GRANULARITY || s.text.length <= TEXT_GRANULARITY) &&
			propsMatch(prev.kv, s.kv)) {
			prev.text += s.text;
			continue;
		}
		out.push({ text: s.text, kv: s.kv, refType: s.refType });
	}
	for (const s of out) if (s.kv && s.kv.length === 0) s.kv = null; // empty props → undefined
	return out;
}

/** toJSONObject: a TextSegment's text or {text, props}; a Marker's {marker: {refType}, props?}. */
function segJsonOf(s, keys, values) {
	const hasProps = s.kv !== null && s.kv !== undefined && s.kv.length > 0;
	if (s.refType !== undefined) {
		const m = { marker: { refType: s.refType } };
		if (hasProps) m.props = propsObject(s.kv, keys, values);
		return m;
	}
	return hasProps ? { text: s.text, props: propsObject(s.kv, keys, values) } : s.text;
}

/** SnapshotLegacy emit: the header chunk (>= sizeOfFirstChunk chars) and the body chunk, if any. */
function legacySummary(segs, minSeq, keys, values, chunkSize) {
	const segments = legacySegments(segs, minSeq);
	const total = segments.reduce((n, s) => n + s.text.length, 0);
	const chunk = (start, approx, isHeader) => {
		let n = 0, length = 0;
		while (length < approx && start + n < segments.length) {
			length += segments[start + n].text.length;
			n++;
		}
		const texts = segments.slice(start, start + n).map((s) => segJsonOf(s, keys, values));
		const j = {
			chunkStartSegmentIndex: start,
			chunkSegmentCount: n,
			chunkLengthChars: length,
			totalLengthChars: total,
			totalSegmentCount: segments.length,
			chunkSequenceNumber: minSeq,
			segmentTexts: texts,
		};
		if (isHeader) {
			const ids = [{ id: "header" }];
			if (length < total) ids.push({ id: "body" });
			j.headerMetadata = {
				orderedChunkMetadata: ids,
				sequenceNumber: minSeq,
				totalLength: total,
				totalSegmentCount: segments.length,
			};
		}
		return [JSON.stringify(j), n];
	};
	const [header, n1] = chunk(0, chunkSize === undefined ? SIZE_OF_FIRST_CHUNK : chunkSize, true);
	const body = n1 < segments.length ? chunk(n1, total, false)[0] : undefined;
	return { header, body };
}

/**
 * SnapshotV1 (newMergeTreeSnapshotFormat; snapshotV1.ts:90-265): every segment above minSeq with its
 * merge info, the rest merged as in extractSync, chunked by SnapshotV1.chunkSize = 10000 lengths.
 * @param segs - leaves in order: {insertSeq, insertClient, removedSeq (or NOT_REMOVED), text, kv}
 * @param removers - {leaf index: [[short client id, seq, kind], ...] of its remove stamps in stamp
 *   order; kind 0 = setRemove, 1 = sliceRemove (obliterate)}
 * @returns {header, bodies} - the blobs "header", "body_0", "body_1", ...
 */
function v1Summary(segs, minSeq, curSeq, keys, values, clientNames, removers, chunkSize) {
	const out = []; // [json value, cachedLength]
	let prev = null;
	const flush = () => {
		if (prev !== null) out.push([segJsonOf(prev, keys, values), prev.text.length]);
	};
	segs.forEach((s, i) => {
		const removed = s.removedSeq !== NOT_REMOVED;
		if (removed && s.removedSeq <= minSeq) return;
		if (s.insertSeq <= minSeq && !removed) {
			if (prev === null) prev = { text: s.text, kv: s.kv, refType: s.refType };
			else if (prev.refType === undefined && s.refType === undefined && !prev.text.endsWith("\n") &&
				(prev.text.length <= TEXT_GRANULARITY || s.text.length <= TEXT_GRANULARITY) &&
				propsMatch(prev.kv, s.kv)) prev = { text: prev.text + s.text, kv: prev.kv };
			else {
				flush();
				prev = { text: s.text, kv: s.kv, refType: s.refType };
			}
			return;
		}
		flush();
		prev = null;
		const raw = { json: segJsonOf(s, keys, values) };
		if (s.insertSeq > minSeq) {
			raw.seq = s.insertSeq;
			raw.client = clientNames[s.insertClient];
		}
		if (removed) {
			const stamps = removers[i];
			if (!stamps || stamps.length === 0) throw new Error(`leaf ${i}: remove order unknown`);
			const sets = stamps.filter((x) => x[2] === 0), moves = stamps.filter((x) => x[2] === 1);
			if (sets.length > 0) { // snapshotV1.ts:235-250
				raw.removedSeq = sets[0][1];
				raw.removedClient = clientNames[sets[0][0]];
				raw.removedClientIds = sets.map((x) => clientNames[x[0]]);
			}
			if (moves.length > 0) { // sliceRemove stamps, "moves" in this format (snapshotV1.ts:252-264)
				raw.movedSeq = moves[0][1];
				raw.movedSeqs = moves.map((x) => x[1]);
				raw.movedClientIds = moves.map((x) => clientNames[x[0]]);
			}
		}
		out.push([raw, s.text.length]);
	});
	flush();
	const size = chunkSize === undefined ? 10000 : chunkSize;
	const chunks = [];
	let start = 0;
	do {
		let n = 0, length = 0;
		while (length < size && start + n < out.length) {
			length += out[start + n][1];
			n++;
		}
		chunks.push({ version: "1", segmentCount: n, length, segments: out.slice(start, start + n).map((x) => x[0]),
			startIndex: start, headerMetadata: undefined });
		start += n;
	} while (start < out.length);
	const header = chunks[0];
	header.headerMetadata = {
		minSequenceNumber: minSeq,
		sequenceNumber: curSeq,
		orderedChunkMetadata: [{ id: "header" }].concat(chunks.slice(1).map((_, k) => ({ id: `body_${k}` }))),
		totalLength: chunks.reduce((n, c) => n + c.length, 0),
		totalSegmentCount: out.length,
	};
	return { header: JSON.stringify(header), bodies: chunks.slice(1).map((c) => JSON.stringify(c)) };
}

/**
 * Catch-up messages (sequence.ts:949-1018): messages after minSeq, transformed ones rebuilt from
 * their delta ranges the way createOpsFromDelta builds them (sequence.ts:395-452).
 * @param messages - [{message, firstOp, count}] as the batch builder kept them.
 * @param ranges - [{op, pos1, pos2, type}] catch-up ranges of the document (engine output).
 */
function insertSegJson(seg) {
	if (typeof seg === "string") return seg;
	if (seg && typeof seg === "object" && "marker" in seg) { // Marker.clone().toJSONObject()
		const m = { marker: { refType: seg.marker.refType } };
		if (seg.props !== undefined && seg.props !== null) {
			m.props = {};
			for (const [k, v] of Object.entries(seg.props)) if (v !== undefined && v !== null) m.props[k] = v;
		}
		return m;
	}
	if (seg.props === undefined || seg.props === null) return seg.text;
	const props = {};
	for (const [k, v] of Object.entries(seg.props)) if (v !== undefined && v !== null) props[k] = v;
	return { text: seg.text, props };
}

function catchupMessages(messages, ranges, minSeq) {
	const byOp = new Map();
	for (const r of ranges) {
		if (!byOp.has(r.op)) byOp.set(r.op, []);
		byOp.get(r.op).push(r);
	}
	const out = [];
	for (const { message, firstOp } of messages) {
		const seq = message.sequenceNumber;
		if (seq <= minSeq) continue;
		let m;
		if (message.referenceSequenceNumber !== seq - 1) {
			const contents = message.contents;
			const members = contents.type === MT_GROUP ? contents.ops : [contents];
			const ops = [];
			members.forEach((op, k) => {
				for (const r of byOp.get(firstOp + k) || []) {
					if (r.type === MT_INSERT) {
						// createInsertOp(pos, segment.clone().toJSONObject()): {text, props} when the
						// segment has properties (textSegment.ts:62-66; clone(props) drops nulls)
						ops.push({ pos1: r.pos1, seg: insertSegJson(op.seg), type: r.type });
					} else if (r.type === MT_REMOVE || r.type === MT_OBLITERATE) {
						// createRemoveRangeOp / createObliterateRangeOp
						ops.push({ pos1: r.pos1, pos2: r.pos2, type: r.type });
					} else {
						ops.push({ pos1: r.pos1, pos2: r.pos2, props: Object.assign({}, op.props || {}), type: r.type });
					}
				}
			});
			m = Object.assign({}, message, {
				referenceSequenceNumber: seq - 1,
				contents: ops.length === 1 ? ops[0] : { ops, type: MT_GROUP },
			});
		} else {
			m = Object.assign({}, message);
		}
		m.minimumSequenceNumber = minSeq;
		delete m.term;
		out.push(m);
	}
	return out;
}

module.exports = { mapSummary, legacySegments, legacySummary, v1Summary, catchupMessages, NOT_REMOVED };
