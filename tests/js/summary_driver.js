"use strict";
// Runs fluidframework_amd/js/summary.js over cases read as JSON from the file argv[2] and prints the
// results as one JSON line. Case kinds:
//   {kind: "string", segs, minSeq, keys, values, messages?, ranges?} → {header, body, catchupOps}
//   {kind: "map", entries}                                           → {header, blobs}
//   {kind: "v1", segs, minSeq, curSeq, keys, values, clients, removers} → {header, bodies}
const fs = require("fs");
const path = require("path");
const summary = require(path.join(__dirname, "..", "..", "fluidframework_amd", "js", "summary.js"));

const cases = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));
const out = cases.map((c) => {
	if (c.kind === "v1") {
		return summary.v1Summary(c.segs, c.minSeq, c.curSeq, c.keys, c.values, c.clients, c.removers);
	}
	if (c.kind === "map") {
		return summary.mapSummary(c.entries.map(([k, v]) => [k, v === null ? undefined : v]));
	}
	const r = summary.legacySummary(c.segs, c.minSeq, c.keys, c.values);
	const res = { header: r.header, body: r.body === undefined ? null : r.body, catchupOps: null };
	if (c.messages) {
		const msgs = summary.catchupMessages(c.messages, c.ranges, c.minSeq);
		if (msgs.length) res.catchupOps = JSON.stringify(msgs);
	}
	return res;
});
process.stdout.write(JSON.stringify(out) + "\n");
