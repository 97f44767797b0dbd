"""Summary emission from the engine's converged state (host side).

  - SharedMap: SharedMap.summarizeCore (packages/dds/map/src/map.ts:176-246) over the key slots
    produced by the map kernel; key order is the JS object order of getSerializedStorage
    (mapKernel.ts:545-551): array-index keys ascending, then Map insertion (birth) order.
  - SharedString legacy format: SnapshotLegacy.extractSync + emit (merge-tree/src/snapshotlegacy.ts:
    74-262, snapshotChunks.ts:85-204) over the leaf table produced by the merge-tree kernel.
  - SharedString SnapshotV1 format (newMergeTreeSnapshotFormat, client.ts:1569-1580):
    SnapshotV1.extractSync + emit (merge-tree/src/snapshotV1.ts:90-265) with merge info for the
    segments above minSeq; removedClientIds come from the kernel's remove-order slab.
Both are byte-identical to JSON.stringify of the reference objects.
"""
from __future__ import annotations

import json

from .native import propset_entries

from .streams import (MAP_ABSENT, MAP_VALUE_UNDEFINED, MT_ANNOTATE, MT_GROUP, MT_INSERT, MT_LEAF_MARKER,
                      MT_OBLITERATE, MT_OBLITERATE_SIDED, MT_REMOVE, VALUE_ADJUST, VALUE_COMPUTED, UnsupportedOp,
                      is_array_index_key, js_json, js_key_order, js_number, js_quote, marker_ref_type)

NOT_REMOVED = 0x7FFFFFFF
TEXT_GRANULARITY = 256          # textSegment.ts:21
SIZE_OF_FIRST_CHUNK = 10000     # snapshotlegacy.ts:55
MIN_VALUE_SIZE_SEPARATE_BLOB = 8 * 1024  # map.ts:190
MAX_SNAPSHOT_BLOB_SIZE = 16 * 1024       # map.ts:194


_q = js_quote  # JSON.stringify of a string (lone surrogates escaped)


def _utf16_len(s: str) -> int:
    return len(s.encode("utf-16-le", "surrogatepass")) // 2


def _js_order(keys):
    idx = sorted((k for k in keys if is_array_index_key(k)), key=int)
    return idx + [k for k in keys if not is_array_index_key(k)]


# ------------------------------------------------------------------------------------------- map
def map_summary(slots, keys, values):
    """(header, [blob0, ...]) for one document's key slots (fmt_map_slot array)."""
    live = [(k, int(s["value"]), int(s["birth_seq"])) for k, s in enumerate(slots) if int(s["value"]) != MAP_ABSENT]
    live.sort(key=lambda t: t[2])  # Map insertion order = birth order
    names = {keys[k]: (v, b) for k, v, b in live}
    order = _js_order([keys[k] for k, _, _ in live])

    def member(name):
        v = names[name][0]
        if v == MAP_VALUE_UNDEFINED:
            return _q(name) + ':{"type":"Plain"}'
        return _q(name) + ':{"type":"Plain","value":' + values[v] + "}"

    blobs, header_members, size = [], [], 0
    for name in order:
        v = names[name][0]
        vlen = 0 if v == MAP_VALUE_UNDEFINED else _utf16_len(values[v])
        if v != MAP_VALUE_UNDEFINED and vlen >= MIN_VALUE_SIZE_SEPARATE_BLOB:
            blobs.append("{" + member(name) + "}")
        else:
            size += len("Plain") + 21 + vlen
            if size > MAX_SNAPSHOT_BLOB_SIZE:
                blobs.append("{" + ",".join(member(m) for m in _js_order(header_members)) + "}")
                header_members, size = [], 0
            header_members.append(name)
    header = (
        '{"blobs":[' + ",".join(_q(f"blob{i}") for i in range(len(blobs))) + '],"content":{'
        + ",".join(member(m) for m in _js_order(header_members)) + "}}"
    )
    return header, blobs


# ------------------------------------------------------------------------------------- merge-tree
def values_with_numbers(values, numbers):
    """The value texts a document's prop sets index: the host dictionary, then the document's
    computed annotate-adjust numbers at FMT_MT_VALUE_COMPUTED + k, written as JSON.stringify writes
    them (ECMAScript Number::toString)."""
    if numbers is None or len(numbers) == 0:
        return values
    return list(values) + [""] * (VALUE_COMPUTED - len(values)) + [js_number(float(x)) for x in numbers]


def _props_obj(kv, keys, values):
    pairs = [(keys[x >> 16], values[x & 0xFFFF]) for x in kv]
    names = [k for k, _ in pairs]
    d = dict(pairs)
    return "{" + ",".join(_q(k) + ":" + d[k] for k in _js_order(names)) + "}"


def _seg_json(text, props, marker, keys, values):
    """toJSONObject of a summary segment (props already normalized: None when undefined or {}):
    a TextSegment's text or {text, props} (textSegment.ts:62-66), a Marker's {marker: {refType},
    props?} (mergeTreeNodes.ts:514-518; its one unit is the refType)."""
    if marker:
        j = '{"marker":{"refType":' + str(ord(text[0]) if isinstance(text, str) else int(text[0])) + "}"
        if props:
            j += ',"props":' + _props_obj(props, keys, values)
        return j + "}"
    if not props:
        return _q(text)
    return '{"text":' + _q(text) + ',"props":' + _props_obj(props, keys, values) + "}"


def _props_match(a, b):
    """properties.ts:32-61 (undefined ≡ {}), on (key, value) id pairs."""
    a, b = a or (), b or ()
    if len(a) != len(b):
        return False
    bd = {x >> 16: x for x in b}
    return all(bd.get(x >> 16) == x for x in a)


def legacy_segments(header, leaves, chars, propsets, min_seq, legacy_props=None):
    """extractSync: leaves present at PriorPerspective(minSeq, NonCollabClient), merged greedily
    (prev.canAppend(seg): both TextSegments; a Marker never appends, mergeTreeNodes.ts:557-559). Each
    leaf's properties are getAtSeq(properties, minSeq) (snapshotlegacy.ts:211-212): for batches with
    annotate-adjust the engine's per-leaf legacy prop sets (legacy_props), else the current ones."""
    segs = []  # [text, props kv tuple or None, marker]
    for i, L in enumerate(leaves[: int(header["n_leaves"])]):
        ins, rm = int(L["ins_seq"]), int(L["rm_seq"])
        if not (ins <= min_seq) or rm <= min_seq:
            continue
        o, n = int(L["char_off"]), int(L["len"])
        text = chars[o : o + n].tobytes().decode("utf-16-le", "surrogatepass")
        marker = (int(L["pad"]) & MT_LEAF_MARKER) != 0
        pid = int(L["props"]) if legacy_props is None else int(legacy_props[i])
        props = None if pid == 0xFFFF else propset_entries(propsets, pid)
        if segs:
            prev = segs[-1]
            if (not prev[2] and not marker and not prev[0].endswith("\n")
                    and (_utf16_len(prev[0]) <= TEXT_GRANULARITY or n <= TEXT_GRANULARITY)
                    and _props_match(prev[1], props)):
                prev[0] += text
                continue
        segs.append([text, props, marker])
    for s in segs:
        if s[1] is not None and len(s[1]) == 0:
            s[1] = None
    return segs


def legacy_summary(header, leaves, chars, propsets, keys, values, chunk_size=SIZE_OF_FIRST_CHUNK, legacy_props=None):
    """(header_blob, body_blob or None) of the legacy SharedString summary at the doc's minSeq
    (legacy_props: the engine's getAtSeq prop set per leaf, batches with annotate-adjust)."""
    min_seq = int(header["min_seq"])
    segs = legacy_segments(header, leaves, chars, propsets, min_seq, legacy_props)
    total_len = sum(_utf16_len(t) for t, _, _ in segs)

    def chunk(start, approx, is_header):
        n, length = 0, 0
        while length < approx and start + n < len(segs):
            length += _utf16_len(segs[start + n][0])
            n += 1
        texts = [_seg_json(t, p, m, keys, values) for t, p, m in segs[start : start + n]]
        j = (
            f'{{"chunkStartSegmentIndex":{start},"chunkSegmentCount":{n},"chunkLengthChars":{length},'
            f'"totalLengthChars":{total_len},"totalSegmentCount":{len(segs)},"chunkSequenceNumber":{min_seq},'
            f'"segmentTexts":[{",".join(texts)}]'
        )
        if is_header:
            ids = '[{"id":"header"}' + (',{"id":"body"}' if length < total_len else "") + "]"
            j += (
                f',"headerMetadata":{{"orderedChunkMetadata":{ids},"sequenceNumber":{min_seq},'
                f'"totalLength":{total_len},"totalSegmentCount":{len(segs)}}}'
            )
        return j + "}", n

    head, n1 = chunk(0, chunk_size, True)
    body = chunk(n1, total_len, False)[0] if n1 < len(segs) else None
    return head, body


# ------------------------------------------------------------------------------ SnapshotV1 (f2)
V1_CHUNK_SIZE = 10000  # SnapshotV1.chunkSize (snapshotV1.ts:44)


def removers_from_engine(leaves, n_leaves, rm_order, doc_ops):
    """Remove stamps per removed leaf, in stamp order: {leaf: [(client, seq, kind), ...]}, kind 0 =
    setRemove, 1 = sliceRemove (stamps.ts RemoveOperationStamp). The first stamp is the op whose seq
    is the leaf's rm_seq (its client, and its type: REMOVE or an obliterate); later ones are the
    kernel's remove-order entries, which carry their own seq and kind (stamps.ts:144-158 keeps remote
    stamps in seq order, so the entries of one leaf are sorted by seq)."""
    first = {}
    for s, c, t in zip(doc_ops["seq"], doc_ops["client"], doc_ops["type"]):
        if int(t) in (MT_REMOVE, MT_OBLITERATE, MT_OBLITERATE_SIDED):
            first.setdefault(int(s), (int(c), 0 if int(t) == MT_REMOVE else 1))
    out = {}
    for i in range(n_leaves):
        rm = int(leaves[i]["rm_seq"])
        if rm != NOT_REMOVED and rm in first:
            c, k = first[rm]
            out[i] = [(c, rm, k)]
    later = {}
    for e in rm_order:
        j = int(e["leaf"])
        if j != 0xFFFFFFFF and j in out:
            later.setdefault(j, []).append((int(e["client"]), int(e["seq"]), int(e["kind"])))
    for j, es in later.items():
        out[j].extend(sorted(es, key=lambda x: x[1]))
    return out


def v1_segments(header, leaves, chars, propsets, keys, values, client_names, removers):
    """SnapshotV1.extractSync (snapshotV1.ts:170-276): [(json text, cachedLength)] per summary segment.
    Leaves removed at/below minSeq are skipped (the merge chain continues across them); acked,
    not-removed leaves at/below minSeq merge while canAppend && matchProperties; every other leaf is
    written with its merge info."""
    min_seq = int(header["min_seq"])
    out = []
    prev = None  # [text, props, marker]

    def seg_json(text, props, marker):
        return _seg_json(text, props or None, marker, keys, values)

    def flush():
        if prev is not None:
            out.append((seg_json(prev[0], prev[1], prev[2]), _utf16_len(prev[0])))

    for i in range(int(header["n_leaves"])):
        L = leaves[i]
        ins, rm = int(L["ins_seq"]), int(L["rm_seq"])
        removed = rm != NOT_REMOVED
        if removed and rm <= min_seq:
            continue
        o, n = int(L["char_off"]), int(L["len"])
        text = chars[o : o + n].tobytes().decode("utf-16-le", "surrogatepass")
        marker = (int(L["pad"]) & MT_LEAF_MARKER) != 0
        pid = int(L["props"])
        props = None if pid == 0xFFFF else propset_entries(propsets, pid)
        if ins <= min_seq and not removed:
            if prev is None:
                prev = [text, props, marker]
            elif (not prev[2] and not marker and not prev[0].endswith("\n")
                  and (_utf16_len(prev[0]) <= TEXT_GRANULARITY or n <= TEXT_GRANULARITY)
                  and _props_match(prev[1], props)):
                prev[0] += text
            else:
                flush()
                prev = [text, props, marker]
            continue
        flush()
        prev = None
        raw = '{"json":' + seg_json(text, props, marker)
        if ins > min_seq:
            raw += f',"seq":{ins},"client":' + _q(client_names[int(L["ins_client"])])
        if removed:
            stamps = removers.get(i)
            if not stamps:
                raise ValueError(f"leaf {i}: remove order unknown (flag removes with FMT_MT_F_RMORDER)")
            sets = [st for st in stamps if st[2] == 0]
            moves = [st for st in stamps if st[2] == 1]
            if sets:  # setRemove stamps (snapshotV1.ts:235-250)
                raw += (f',"removedSeq":{sets[0][1]},"removedClient":' + _q(client_names[sets[0][0]])
                        + ',"removedClientIds":[' + ",".join(_q(client_names[st[0]]) for st in sets) + "]")
            if moves:  # sliceRemove stamps: "moves" in this format (snapshotV1.ts:252-264)
                raw += (f',"movedSeq":{moves[0][1]},"movedSeqs":[' + ",".join(str(st[1]) for st in moves)
                        + '],"movedClientIds":[' + ",".join(_q(client_names[st[0]]) for st in moves) + "]")
        out.append((raw + "}", n))
    flush()
    return out


def v1_summary(header, leaves, chars, propsets, keys, values, client_names, removers,
               chunk_size=V1_CHUNK_SIZE):
    """(header_blob, [body_0, body_1, ...]) of SnapshotV1.emit (snapshotV1.ts:126-168)."""
    segs = v1_segments(header, leaves, chars, propsets, keys, values, client_names, removers)
    chunks = []  # (start, count, length)
    start = 0
    while True:  # do { ... } while (totalSegmentCount < segments.length)
        n, length = 0, 0
        while length < chunk_size and start + n < len(segs):
            length += segs[start + n][1]
            n += 1
        chunks.append((start, n, length))
        start += n
        if start >= len(segs):
            break
    total_len = sum(c[2] for c in chunks)

    def body_of(c):
        s0, n, length = c
        return (f'{{"version":"1","segmentCount":{n},"length":{length},"segments":['
                + ",".join(t for t, _ in segs[s0 : s0 + n]) + f'],"startIndex":{s0}')

    ids = ",".join(['{"id":"header"}'] + [f'{{"id":"body_{k}"}}' for k in range(len(chunks) - 1)])
    head = (body_of(chunks[0]) + f',"headerMetadata":{{"minSequenceNumber":{int(header["min_seq"])},'
            f'"sequenceNumber":{int(header["cur_seq"])},"orderedChunkMetadata":[{ids}],'
            f'"totalLength":{total_len},"totalSegmentCount":{len(segs)}}}}}')
    return head, [body_of(c) + "}" for c in chunks[1:]]


def _insert_seg_json(seg):
    """toJSONObject of the inserted segment's clone: a TextSegment's text, or {text, props} when it
    has properties (textSegment.ts:62-66; clone(props) drops null values, properties.ts:68-95); a
    Marker's {marker: {refType}, props?} (mergeTreeNodes.ts:514-518)."""
    if isinstance(seg, str):
        return seg
    if marker_ref_type(seg) is not None:
        out = {"marker": {"refType": seg["marker"]["refType"]}}
        props = seg.get("props")
        if props is not None:
            out["props"] = {k: props[k] for k in js_key_order(list(props)) if props[k] is not None}
        return out
    props = seg.get("props")
    if props is None:
        return seg["text"]
    return {"text": seg["text"], "props": {k: props[k] for k in js_key_order(list(props)) if props[k] is not None}}


def catchup_messages(messages, ranges, min_seq):
    """The legacy summary's catch-up messages for one document (sequence.ts:949-1018).

    messages: [(message dict as applyMsg received it, first op index, member count)] in order
    (MergeTreeBatch.messages[d]); ranges: the document's fmt_mt_catchup_range records (engine or
    oracle) for its FMT_MT_F_CATCHUP ops; min_seq: the summary's minimumSequenceNumber.
    Messages with seq <= min_seq are dropped (processMinSequenceNumberChanged); a message with
    refSeq == seq - 1 is kept as it is; any other is a shallow copy with refSeq = seq - 1 and
    contents regenerated from its delta ranges by createOpsFromDelta (sequence.ts:395-452): one op
    stays bare, several (or none) become a GROUP op. Every kept message gets minimumSequenceNumber
    = min_seq and loses `term` (sequence.ts:955-957, snapshotlegacy.ts:178-185).
    """
    by_op: dict[int, list] = {}
    for r in ranges:
        by_op.setdefault(int(r["op"]), []).append((int(r["type"]), int(r["pos1"]), int(r["pos2"])))
    out = []
    for msg, first, count in messages:
        seq = int(msg["sequenceNumber"])
        if seq <= min_seq:
            continue
        if int(msg["referenceSequenceNumber"]) != seq - 1:
            contents = msg["contents"]
            members = contents["ops"] if contents["type"] == MT_GROUP else [contents]
            ops = []
            for k, op in enumerate(members):
                for t, p1, p2 in by_op.get(first + k, []):
                    if t == MT_INSERT:  # createInsertOp(pos, segment.clone().toJSONObject())
                        ops.append({"pos1": p1, "seg": _insert_seg_json(op["seg"]), "type": t})
                    elif t in (MT_REMOVE, MT_OBLITERATE):  # createRemoveRangeOp / createObliterateRangeOp
                        ops.append({"pos1": p1, "pos2": p2, "type": t})
                    else:  # createAnnotateRangeOp(pos1, pos2, {...props}): the segment's value ?? null
                        props = op.get("props") or {}
                        ops.append({"pos1": p1, "pos2": p2, "props": {k2: props[k2] for k2 in js_key_order(list(props))},
                                    "type": t})
            msg = dict(msg)
            msg["referenceSequenceNumber"] = seq - 1
            msg["contents"] = ops[0] if len(ops) == 1 else {"ops": ops, "type": MT_GROUP}
        else:
            msg = dict(msg)
        msg["minimumSequenceNumber"] = min_seq
        msg.pop("term", None)
        out.append(msg)
    return out


def catchup_blob(msgs):
    """JSON.stringify(catchUpMsgs) (snapshotlegacy.ts:186-189), or None when there are none."""
    if not msgs:
        return None
    return js_json(msgs)


def bulk_catchup_blobs(messages, min_seqs, offsets, ranges):
    """The catchupOps blob (or None) of every document from one bulk fetch of the catch-up ranges
    (Engine.mt_catchup_all: offsets[n_docs + 1], ranges): what summarizeMergeTree emits for each
    string (sequence.ts:949-964, snapshotlegacy.ts:178-190). messages[d]: the batch's kept messages."""
    out = []
    for d, msgs in enumerate(messages):
        if not msgs:
            out.append(None)
            continue
        r = ranges[int(offsets[d]) : int(offsets[d + 1])]
        out.append(catchup_blob(catchup_messages(msgs, r, int(min_seqs[d]))))
    return out


def summary_tree(header_blob, body_blob, catchup=None):
    """convertSummaryTreeToITree shape of SharedString.summarizeCore's content subtree (blobs in
    SnapshotLegacy.emit order: header, body, catchupOps)."""
    entries = [{"path": "header", "mode": "100644", "type": "Blob",
                "value": {"contents": header_blob, "encoding": "utf-8"}}]
    if body_blob is not None:
        entries.append({"path": "body", "mode": "100644", "type": "Blob",
                        "value": {"contents": body_blob, "encoding": "utf-8"}})
    if catchup is not None:
        entries.append({"path": "catchupOps", "mode": "100644", "type": "Blob",
                        "value": {"contents": catchup, "encoding": "utf-8"}})
    return {"entries": [{"path": "content", "mode": "040000", "type": "Tree", "value": {"entries": entries}}]}


def dumps_tree(tree) -> str:
    return json.dumps(tree, indent=1)
