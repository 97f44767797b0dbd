"use strict";
// Drives fluidframework_amd/js/fmt.js over the reference's replay fixtures
// (tests/golden/replay_msgs_0.40.json.gz; client.replay.spec.ts:20-76 replays the same messages).
//
//   node fixture_driver.js pack <outdir>   pack every fixture (one document per checkpoint prefix) and
//                                          write the raw buffers for the Python packer comparison (CPU)
//   node fixture_driver.js replay          replay them on the GPU through the N-API addon and print
//                                          {"checked": n, "mismatches": [...]} as one JSON line
//   node fixture_driver.js map             a SharedMap bunch replay through processMessagesCore (GPU)
//   node fixture_driver.js summary         legacy summaries + catch-up blobs of each fixture (GPU)
//   node fixture_driver.js v1              SnapshotV1 summaries of each fixture (GPU)
const fs = require("fs");
const path = require("path");
const zlib = require("zlib");
const fmt = require(path.join(__dirname, "..", "..", "fluidframework_amd", "js", "fmt.js"));

const GOLDEN = path.join(__dirname, "..", "golden", "replay_msgs_0.40.json.gz");

function loadFixtures() {
	return JSON.parse(zlib.gunzipSync(fs.readFileSync(GOLDEN)).toString("utf8"));
}

/** Document k of a fixture replays groups 0..k (initial text of group 0), expecting resultText of k. */
function buildBatch(fixtures, stride) {
	const b = new fmt.MergeTreeStreamBuilder();
	const expected = [];
	for (const fx of fixtures) {
		const groups = fx.groups;
		for (let k = 0; k < groups.length; k += stride) {
			const doc = b.beginDoc(groups[0].initialText, "A");
			for (let g = 0; g <= k; g++) {
				for (const m of groups[g].msgs) doc.addMessage(m);
			}
			expected.push({ name: fx.name, group: k, text: groups[k].resultText });
		}
	}
	return { batch: b.finish(), expected };
}

async function replay() {
	const fixtures = loadFixtures();
	const { batch, expected } = buildBatch(fixtures, 1);
	const eng = new fmt.Engine(0);
	try {
		const t0 = Date.now();
		const r = await eng.replayMergeTree(batch);
		const ms = Date.now() - t0;
		const mismatches = [];
		expected.forEach((e, d) => {
			const got = r.getText(d);
			if (got !== e.text) mismatches.push({ doc: d, name: e.name, group: e.group, got, want: e.text });
		});
		console.log(JSON.stringify({ checked: expected.length, mismatches: mismatches.slice(0, 5),
			nMismatches: mismatches.length, device: eng.deviceInfo(), ms }));
	} finally {
		eng.close();
	}
}

function pack(outdir) {
	const fixtures = loadFixtures();
	const { batch, expected } = buildBatch(fixtures, 8);
	fs.mkdirSync(outdir, { recursive: true });
	const w = (name, arr) => fs.writeFileSync(path.join(outdir, name),
		Buffer.from(arr.buffer, arr.byteOffset, arr.byteLength));
	w("ops.bin", batch.ops);
	w("offs.bin", batch.docOpOffsets);
	w("text.bin", batch.text);
	w("doc_init.bin", batch.docInit);
	w("props_off.bin", batch.propsOff);
	w("props_kv.bin", batch.propsKv);
	fs.writeFileSync(path.join(outdir, "meta.json"), JSON.stringify({
		keys: batch.keys, values: batch.values, clients: batch.clients, expected }));
}

/** SharedMap: bunches through processMessagesCore, then entries()/get() against the LWW rule. */
async function mapDemo() {
	const b = new fmt.MapStreamBuilder();
	const d0 = b.beginDoc();
	const env = (seq) => ({ envelope: { sequenceNumber: seq, clientId: "A", type: "op" }, local: false });
	b.processMessagesCore(d0, Object.assign(env(1), { messagesContent: [
		{ contents: { type: "set", key: "b", value: { type: "Plain", value: 1 } }, clientSequenceNumber: 1 },
		{ contents: { type: "set", key: "a", value: { type: "Plain", value: "x" } }, clientSequenceNumber: 2 },
	] }));
	b.processMessagesCore(d0, Object.assign(env(2), { messagesContent: [
		{ contents: { type: "delete", key: "b" }, clientSequenceNumber: 3 },
		{ contents: { type: "set", key: "b", value: { type: "Plain", value: { n: [1, 2] } } }, clientSequenceNumber: 4 },
		{ contents: { type: "set", key: "a", value: { type: "Plain", value: "y" } }, clientSequenceNumber: 5 },
	] }));
	const d1 = b.beginDoc();
	b.processMessagesCore(d1, Object.assign(env(1), { messagesContent: [
		{ contents: { type: "set", key: "a", value: { type: "Plain" } }, clientSequenceNumber: 1 },
		{ contents: { type: "clear" }, clientSequenceNumber: 2 },
		{ contents: { type: "set", key: "c", value: { type: "Plain", value: true } }, clientSequenceNumber: 3 },
	] }));
	const batch = b.finish();
	const eng = new fmt.Engine(0);
	try {
		const r = await eng.replayMap(batch);
		console.log(JSON.stringify({ doc0: r.entries(0), doc1: r.entries(1), a0: r.get(0, "a"),
			summary0: r.summarize(0).header }));
	} finally {
		eng.close();
	}
}

/** Legacy summaries (with catch-up blobs) of each fixture's final state, from GPU state. */
async function summaries() {
	const fixtures = loadFixtures();
	const b = new fmt.MergeTreeStreamBuilder({ keepMessages: true });
	for (const fx of fixtures) {
		const doc = b.beginDoc(fx.groups[0].initialText, "A");
		for (const g of fx.groups) for (const m of g.msgs) doc.addMessage(m);
	}
	const batch = b.finish({ catchup: true });
	const eng = new fmt.Engine(0);
	try {
		const r = await eng.replayMergeTree(batch);
		const out = fixtures.map((fx, d) => {
			const s = r.summarize(d);
			return { header: s.header, body: s.body === undefined ? null : s.body,
				catchupOps: s.catchupOps === undefined ? null : s.catchupOps };
		});
		console.log(JSON.stringify(out));
	} finally {
		eng.close();
	}
}

/** SnapshotV1 summaries of each fixture's final state from GPU state (remove order recorded). */
async function summariesV1() {
	const fixtures = loadFixtures();
	const b = new fmt.MergeTreeStreamBuilder();
	for (const fx of fixtures) {
		const doc = b.beginDoc(fx.groups[0].initialText, "A");
		for (const g of fx.groups) for (const m of g.msgs) doc.addMessage(m);
	}
	const batch = b.finish({ removeOrder: true });
	const eng = new fmt.Engine(0);
	try {
		const r = await eng.replayMergeTree(batch);
		console.log(JSON.stringify(fixtures.map((fx, d) => r.summarizeV1(d))));
	} finally {
		eng.close();
	}
}

/** Pack documents loaded from summaries ([[header, body, catchupOps], ...] in argv[3]) into argv[4]. */
function packSummaries(input, outdir) {
	const sums = JSON.parse(fs.readFileSync(input, "utf8"));
	const b = new fmt.MergeTreeStreamBuilder();
	for (const [h, body, cu] of sums) b.beginDocFromSummary(h, body, cu);
	const batch = b.finish();
	fs.mkdirSync(outdir, { recursive: true });
	const w = (name, arr) => fs.writeFileSync(path.join(outdir, name),
		Buffer.from(arr.buffer, arr.byteOffset, arr.byteLength));
	w("ops.bin", batch.ops);
	w("text.bin", batch.text);
	w("snapshots.bin", new Uint8Array(batch.snapshots));
	w("snapshot_segs.bin", batch.snapshotSegs);
	w("props_kv.bin", batch.propsKv);
}

const mode = process.argv[2];
if (mode === "pack") {
	pack(process.argv[3]);
} else if (mode === "replay") {
	replay().catch((e) => { console.error(e); process.exit(1); });
} else if (mode === "packsummaries") {
	packSummaries(process.argv[3], process.argv[4]);
} else if (mode === "summary") {
	summaries().catch((e) => { console.error(e); process.exit(1); });
} else if (mode === "v1") {
	summariesV1().catch((e) => { console.error(e); process.exit(1); });
} else if (mode === "map") {
	mapDemo().catch((e) => { console.error(e); process.exit(1); });
} else {
	console.error("usage: fixture_driver.js pack <outdir> | replay | summary | map");
	process.exit(2);
}
