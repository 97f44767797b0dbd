"""Host driver: pack sequenced Fluid messages into the engine's SoA op buffers.

This is the batching half of the drop-in boundary. The reference handles one message at a time in
`SharedObject.processMessages` (packages/dds/shared-object-base/src/sharedObject.ts:605-650) and
flags that granularity itself as a performance problem (sharedObject.ts:411-413). Here a batch of
documents' messages is packed once into the 32-byte `fmt_mt_op` / 16-byte `fmt_map_op` records of
include/fmt.h plus a UTF-16 text arena and a props-op table, and crosses host→HBM in one copy.

Semantics mirrored while packing:
  - short client ids are interned per document in order of first appearance, the observer first,
    a missing clientId is "server" (client.ts:831-855, getOrAddShortClientIdFromMessage);
  - GROUP messages are flattened into member records that share the message's seq
    (client.ts:1311-1319 applyRemoteOp GROUP branch; updateSeqNumbers runs once per message);
  - annotate props keep JS object key order (array-index keys first, ascending) because
    `Object.entries(op.props)` drives application order (segmentPropertiesManager.ts:80-88);
  - values are re-serialized the way the summary does: JSON.stringify(JSON.parse(v)).
"""
from __future__ import annotations

import json
from decimal import Decimal
from dataclasses import dataclass, field

import numpy as np

# include/fmt.h fmt_mt_op (32 bytes)
MT_OP_DTYPE = np.dtype(
    [
        ("seq", "<i4"),
        ("ref_seq", "<i4"),
        ("min_seq", "<i4"),
        ("pos1", "<i4"),
        ("pos2", "<i4"),
        ("payload", "<u4"),
        ("len", "<u2"),
        ("client", "u1"),
        ("type", "u1"),
        ("flags", "<u4"),
    ]
)
assert MT_OP_DTYPE.itemsize == 32

# include/fmt.h fmt_mt_snapshot_doc (32 bytes) / fmt_mt_snapshot_seg (12 bytes)
SNAPSHOT_DOC_DTYPE = np.dtype([("first_seg", "<u8"), ("n_header", "<u4"), ("n_body", "<u4"),
                               ("min_seq", "<i4"), ("seq", "<i4"), ("loaded", "<u4"), ("pad", "<u4")])
assert SNAPSHOT_DOC_DTYPE.itemsize == 32
SNAPSHOT_SEG_DTYPE = np.dtype([("text", "<u4"), ("len", "<u4"), ("props", "<u4")])
# fmt_mt_snapshot_info / fmt_mt_stamp: SnapshotV1 merge info of loaded header segments
SNAPSHOT_INFO_DTYPE = np.dtype([("ins_seq", "<i4"), ("ins_client", "<i4"), ("rm_first", "<u4"), ("rm_count", "<u4")])
STAMP_DTYPE = np.dtype([("seq", "<i4"), ("client", "<i4"), ("kind", "<u4"), ("pad", "<u4")])
NON_COLLAB_CLIENT = -2  # fmt.h FMT_NON_COLLAB_CLIENT
assert SNAPSHOT_SEG_DTYPE.itemsize == 12
NO_PROPS = 0xFFFFFFFF

# include/fmt.h fmt_map_op (16 bytes)
MAP_OP_DTYPE = np.dtype([("doc", "<u4"), ("key", "<u4"), ("seq", "<u4"), ("kind_value", "<u4")])
# fmt.h fmt_map_local_op: one event of a document's local client (FMT_MAP_EV_*)
MAP_LOCAL_OP_DTYPE = np.dtype([("doc", "<u4"), ("key", "<u4"), ("event", "<u4"), ("kind_value", "<u4")])
MAP_EV_SUBMIT, MAP_EV_ACK, MAP_EV_ROLLBACK = 0, 1, 2
MAP_PENDING_BIRTH = 0x80000000
assert MAP_OP_DTYPE.itemsize == 16

MT_INSERT, MT_REMOVE, MT_ANNOTATE, MT_GROUP, MT_OBLITERATE, MT_OBLITERATE_SIDED = range(6)
MT_F_START_BEFORE, MT_F_END_BEFORE = 8, 16  # fmt.h FMT_MT_F_START_BEFORE / FMT_MT_F_END_BEFORE
MT_F_MARKER = 32  # fmt.h FMT_MT_F_MARKER: insert of a Marker segment
MT_F_REL1, MT_F_REL2 = 64, 128  # fmt.h FMT_MT_F_REL1/REL2: pos1/pos2 index the relpos table
MT_F_LOADSEG = 256  # fmt.h FMT_MT_F_LOADSEG: a SnapshotV1 body segment the loader appends
MT_F_LEN_HI_SHIFT, MT_F_LEN_HI_MASK = 16, 0x00FF0000  # fmt.h: bits 16..23 of an insert's length
# fmt.h f4, the local client: a submission, the ack of the oldest pending op, rollback of the newest,
# reconnect (regeneratePendingOp for every pending op)
MT_F_LOCAL, MT_F_ACK, MT_F_ROLLBACK, MT_F_REGEN = 512, 1024, 2048, 4096
MT_F_LOCAL_ANY = MT_F_LOCAL | MT_F_ACK | MT_F_ROLLBACK | MT_F_REGEN
LOCAL_SEQ_BASE = 0x40000000  # fmt.h FMT_MT_LOCAL_SEQ_BASE: ins_seq / rm_seq of a stamp pending its ack
MAX_INSERT_UNITS = (1 << 24) - 1


def op_len(rec) -> int:
    """The full length of a packed INSERT record (fmt.h fmt_mt_op_len)."""
    return int(rec["len"]) | (int(rec["flags"]) & MT_F_LEN_HI_MASK)
CLIENT_NONCOLLAB_OP = 0xFE  # fmt.h FMT_MT_CLIENT_NONCOLLAB
# fmt_mt_relpos: an IRelativePosition {id, before, offset} (ops.ts IRelativePosition)
RELPOS_DTYPE = np.dtype([("marker_id", "<u4"), ("offset", "<i4"), ("flags", "<u4"), ("pad", "<u4")])
NO_MARKER = 0xFFFFFFFF  # fmt.h FMT_MT_NO_MARKER
REL_BEFORE = 1  # fmt.h FMT_MT_REL_BEFORE
MARKER_ID_KEY = "markerId"  # reservedMarkerIdKey (merge-tree/src/ops.ts)
MT_SEG_MARKER = 0x80000000  # fmt.h FMT_MT_SEG_MARKER (snapshot segment len flag)
# annotate-adjust (fmt.h): props_kv escape, computed value ids, fmt_mt_adjust rows and their flags
VALUE_ADJUST, VALUE_COMPUTED = 0xFFFF, 0x8000
ADJ_MIN, ADJ_MIN_NULL, ADJ_MAX, ADJ_MAX_NULL = 1, 2, 4, 8
ADJUST_DTYPE = np.dtype([("delta", "<f8"), ("min", "<f8"), ("max", "<f8"), ("flags", "<u4"), ("pad", "<u4")])


def value_numbers(values) -> np.ndarray:
    """Per value JSON text: its number (JSON.parse gives typeof "number"), else NaN."""
    out = np.full(len(values), np.nan)
    for i, t in enumerate(values):
        try:
            v = json.loads(t)
        except ValueError:
            continue
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            out[i] = float(v)
    return out
MT_LEAF_MARKER = 0x8000  # fmt.h FMT_MT_LEAF_MARKER (fmt_mt_leaf.pad flag)


def marker_ref_type(spec) -> int | None:
    """The refType of a Marker segment spec {\"marker\": {\"refType\"}, \"props\"?} (IJSONMarkerSegment,
    mergeTreeNodes.ts:514-525), or None when `spec` is not a marker."""
    if not (isinstance(spec, dict) and "marker" in spec):
        return None
    if not set(spec) <= {"marker", "props"} or not isinstance(spec["marker"], dict):
        raise UnsupportedOp("marker spec")
    ref = spec["marker"].get("refType")
    if not isinstance(ref, int) or isinstance(ref, bool) or not 0 <= ref <= 0xFFFF:
        raise UnsupportedOp("marker refType")
    return ref
MT_F_GROUP_CONT = 1
MT_F_CATCHUP = 2  # include/fmt.h FMT_MT_F_CATCHUP
MT_F_RMORDER = 4  # include/fmt.h FMT_MT_F_RMORDER
MAP_SET, MAP_DELETE, MAP_CLEAR = 0, 1, 2
MAP_KIND_SHIFT = 30
MAP_VALUE_UNDEFINED = 0x3FFFFFFF
MAP_ABSENT = 0xFFFFFFFF
MAX_CLIENTS = 253  # short ids 1..253 (the observer is 0; 0xFE names NonCollab): the small tier keeps 31 writers,
# the large 63, the huge tier 253 (two mask words per leaf plus a side table for ids 64..253); documents
# grow to fit
# Short ids up to 31 (the small tier's writers) are handed out fresh; past that a new client takes the
# id of a client whose every stamp is at or below the engine's minSeq (see _DocBuilder.short_client).
RECYCLE_FROM = 32


class UnsupportedOp(NotImplementedError):
    """An op kind outside the engine's current scope (FMT_E_UNSUPPORTED)."""


def is_array_index_key(k: str) -> bool:
    """CanonicalNumericIndexString for array indices (JS enumerates these keys first)."""
    if not k or len(k) > 10 or (len(k) > 1 and k[0] == "0") or not k.isdigit():
        return False
    return int(k) < 4294967295


def js_key_order(keys):
    """OrdinaryOwnPropertyKeys order of a plain object built with `keys` in insertion order."""
    idx = sorted((k for k in keys if is_array_index_key(k)), key=int)
    return idx + [k for k in keys if not is_array_index_key(k)]


_JS_ESC = {'"': '\\"', "\\": "\\\\", "\b": "\\b", "\f": "\\f", "\n": "\\n", "\r": "\\r", "\t": "\\t"}


def js_quote(s: str) -> str:
    """JSON.stringify of a string (ECMAScript QuoteJSONString, well-formed JSON.stringify: lone
    surrogates are escaped as \\udXXX, which json.dumps(ensure_ascii=False) would write raw)."""
    out = ['"']
    for ch in s:
        c = ord(ch)
        e = _JS_ESC.get(ch)
        if e is not None:
            out.append(e)
        elif c < 0x20 or 0xD800 <= c <= 0xDFFF:
            out.append("\\u%04x" % c)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def js_json(value) -> str:
    """JSON.stringify for JSON-parsed values (ints, strings, bools, null, arrays, objects)."""
    if isinstance(value, dict):
        return "{" + ",".join(
            js_quote(k) + ":" + js_json(value[k]) for k in js_key_order(list(value))
        ) + "}"
    if isinstance(value, list):
        return "[" + ",".join(js_json(v) for v in value) + "]"
    if isinstance(value, str):
        return js_quote(value)
    if isinstance(value, bool) or value is None:
        return json.dumps(value)
    if isinstance(value, int):  # JSON.parse reads every number as a double
        return str(value) if abs(value) <= 2**53 else js_number(float(value))
    if isinstance(value, float):
        return js_number(value)
    raise TypeError(f"not a JSON value: {value!r}")


def js_number(x: float) -> str:
    """JSON.stringify of a JS number: ECMAScript Number::toString (ECMA-262 §6.1.6.1.20) over the
    shortest round-trip digits (which Python's repr also picks), "null" for NaN / ±Infinity
    (SerializeJSONProperty), and "0" for -0."""
    if x != x or x in (float("inf"), float("-inf")):
        return "null"
    if x == 0:
        return "0"
    if x < 0:
        return "-" + js_number(-x)
    sign, digits, exp = Decimal(repr(x)).as_tuple()
    ds = "".join(map(str, digits)).rstrip("0")
    exp += len(digits) - len(ds)  # x = int(ds) × 10^exp
    k = len(ds)
    n = k + exp  # x = 0.ds × 10^n
    if k <= n <= 21:
        return ds + "0" * (n - k)
    if 0 < n <= 21:
        return ds[:n] + "." + ds[n:]
    if -6 < n <= 0:
        return "0." + "0" * (-n) + ds
    e = n - 1
    es = ("+" if e >= 0 else "-") + str(abs(e))
    return (ds if k == 1 else ds[0] + "." + ds[1:]) + "e" + es


def utf16(text: str) -> np.ndarray:
    return np.frombuffer(text.encode("utf-16-le", "surrogatepass"), dtype="<u2")


class Dictionary:
    """Interns strings to dense ids (first come, first served)."""

    def __init__(self, reserved=()):
        self.items: list[str] = list(reserved)
        self.ids: dict[str, int] = {s: i for i, s in enumerate(self.items)}

    def intern(self, s: str) -> int:
        i = self.ids.get(s)
        if i is None:
            i = len(self.items)
            self.items.append(s)
            self.ids[s] = i
        return i


@dataclass
class MergeTreeBatch:
    ops: np.ndarray          # MT_OP_DTYPE
    doc_op_offsets: np.ndarray  # uint64, n_docs + 1
    text: np.ndarray         # uint16 arena
    doc_init: np.ndarray     # uint32 (n_docs, 2): initial text (offset, len)
    props_off: np.ndarray    # uint32, n_props_ops + 1
    props_kv: np.ndarray     # uint32 (key << 16) | value, value 0 = null
    keys: list               # key id → key string
    values: list             # value id → JSON text ("null" at id 0, meaning delete)
    clients: list = field(default_factory=list)  # per doc: short id → long client id
    # per doc (only with keep_messages): [(message dict as applyMsg received it, first op index in
    # the doc, member op count)] — what SharedSegmentSequence stashes for catch-up ops
    messages: list = field(default_factory=list)
    # optional (f3): per-doc fmt_mt_snapshot_doc and the segment specs they index
    snapshots: np.ndarray | None = None
    snapshot_segs: np.ndarray | None = None
    # optional (legacy relativePos1/2): RELPOS_DTYPE table and the key id of "markerId"
    relpos: np.ndarray | None = None
    marker_id_key: int = NO_MARKER
    # optional (SnapshotV1 merge info): per snapshot segment SNAPSHOT_INFO_DTYPE, and the stamps
    snapshot_info: np.ndarray | None = None
    snapshot_stamps: np.ndarray | None = None
    # optional (annotate-adjust): ADJUST_DTYPE rows and, per value id, the number its text holds (NaN)
    adjusts: np.ndarray | None = None
    value_num: np.ndarray | None = None
    # optional (fmt.h doc_value_base): document-local value ids — value id v >= 1 of document d names
    # values[value_base[d] + v]; None: ids are batch-global
    value_base: np.ndarray | None = None

    @property
    def n_docs(self) -> int:
        return len(self.doc_op_offsets) - 1

    def doc_values(self, d: int):
        """Document d's value table: its value id → JSON text (the batch's table when ids are global)."""
        if self.value_base is None:
            return self.values
        b0, b1 = int(self.value_base[d]), int(self.value_base[d + 1])
        return ["null"] + self.values[b0 + 1 : b1 + 1]


class _DocBuilder:
    def __init__(self, owner: "MergeTreeStreamBuilder", observer: str):
        self.owner = owner
        self.client_ids = {observer: 0}
        self.client_names = [observer]
        self.last_stamp = [None]  # per short id: the current holder's latest stamp seq (None: none yet)
        self.min_seq = 0          # the engine's minSeq when the next message applies
        self.ops: list[tuple] = []
        self.messages: list[tuple] = []
        # idToMarker history (mergeTree.ts:675, 1614-1620, 2835-2840; zamboni.ts:202-204): the engine
        # finds a relative position's marker by the "markerId" its leaf holds now, which is the
        # reference's map as long as every id names one marker and no annotate rewrites an id
        self.marker_ids: set = set()
        self.marker_ambiguous = False
        self.uses_relpos = False
        # f4: the local client (the observer name is its long id, short id 0). pending: its
        # unacknowledged ops in submission order, each (record type, payload) — what ACK and
        # ROLLBACK records must repeat (mergeTree.ts:1325-1408, 2388-2514)
        self.local = False
        self.pending: list[tuple] = []  # (record type, payload, refSeq)
        self.regen_ref = 0  # the oldest refSeq among the ops the last reconnect regenerated
        self.cur_seq = 0  # the last message's seq: a local op's refSeq (sequence.ts:666 currentRefSeq)

    def note_marker_id(self, props) -> None:
        mid = (props or {}).get(MARKER_ID_KEY)
        if mid:
            k = js_json(mid)
            self.marker_ambiguous |= k in self.marker_ids
            self.marker_ids.add(k)
            self._check_markers()

    def _check_markers(self) -> None:
        if self.uses_relpos and self.marker_ambiguous:
            raise UnsupportedOp("relative positions in a document whose marker ids repeat or are re-annotated")

    def _note_op(self, op) -> None:
        if op is None:
            return
        t = op.get("type")
        if t == MT_INSERT and marker_ref_type(op.get("seg")) is not None:
            self.note_marker_id(op["seg"].get("props"))
        if t == MT_ANNOTATE and MARKER_ID_KEY in (op.get("props") or {}):
            self.marker_ambiguous = True
        if ((op.get("pos1") is None and op.get("relativePos1") is not None)
                or (op.get("pos2") is None and op.get("relativePos2") is not None)):
            self.uses_relpos = True
        self._check_markers()

    @property
    def n_ops(self) -> int:
        return len(self.ops)

    def short_client(self, long_id, seq=None) -> int:
        """The short id of a long client id (getOrAddShortClientId, client.ts:831-855), noting a
        stamp at `seq`. The reference never forgets a long id; here ids are recycled, because every
        reconnect brings a new clientId and the engine's remove-client sets hold 31 (small tier), 63
        (large tier) or 253 (huge tier) writers. A short id matters only through stamps above minSeq: a perspective
        (refSeq >= minSeq, client) sees a stamp at or below minSeq by its seq whoever made it, and
        merge info (SnapshotV1, catch-up) is written only for stamps above the final minSeq. So once
        every stamp of a client is at or below the engine's minSeq, its id can pass to a new client
        (a returning client just gets a new id). Ids stay fresh up to RECYCLE_FROM - 1; the oldest
        free-able id is taken before a fresh one past that. After the last op, client_names[id] is
        the name of every stamp above the final minSeq that carries the id."""
        long_id = "server" if long_id is None else long_id
        i = self.client_ids.get(long_id)
        if i is None:
            i = len(self.client_names)
            if i >= RECYCLE_FROM:
                # the engine's minSeq: in a document with local events it is also bounded by the
                # oldest pending op's refSeq (getMinInFlightRefSeq, client.ts:1374-1378)
                floor = min([self.min_seq] + [p[2] for p in self.pending])
                for j in range(1, len(self.client_names)):
                    st = self.last_stamp[j]
                    if st is None or st <= floor:
                        del self.client_ids[self.client_names[j]]
                        self.client_names[j] = long_id
                        self.last_stamp[j] = None
                        i = j
                        break
            if i == len(self.client_names):
                if i > MAX_CLIENTS:
                    raise UnsupportedOp(f"more than {MAX_CLIENTS} clients with stamps above minSeq in one document")
                self.client_names.append(long_id)
                self.last_stamp.append(None)
            self.client_ids[long_id] = i
        if seq is not None and (self.last_stamp[i] is None or seq > self.last_stamp[i]):
            self.last_stamp[i] = seq
        return i

    def add_message(self, msg: dict) -> None:
        """Append one ISequencedDocumentMessage (type "op") with merge-tree contents. In a document
        with local events (f4), a message of the local client itself acknowledges its oldest pending
        ops, one per member (client.ts:1367-1368 ackPendingSegment)."""
        seq = int(msg["sequenceNumber"])
        ref = int(msg["referenceSequenceNumber"])
        msn = int(msg["minimumSequenceNumber"])
        client = self.short_client(msg.get("clientId"), seq)
        contents = msg["contents"]
        members = contents["ops"] if contents["type"] == MT_GROUP else [contents]
        if not members:
            members = [None]
        ack = self.local and client == 0
        if self.owner.keep_messages:
            self.messages.append((msg, len(self.ops), len(members)))
        for k, op in enumerate(members):
            if not ack:  # (an ack repeats the local op noted at its submission: the same marker)
                self._note_op(op)
            rec = self.owner._pack(op, seq, ref, msn, client)
            if k > 0:  # later members of a GROUP message (FMT_MT_F_GROUP_CONT)
                rec = rec[:-1] + (rec[-1] | 1,)
            if ack:
                if op is None or not self.pending or self.pending[0][0] != rec[8]:
                    raise ValueError("an ack that is not the oldest pending local op")  # mergeTree.ts:1331-1340
                self.pending.pop(0)
                rec = rec[:-1] + (rec[-1] | MT_F_ACK,)
            self.ops.append(rec)
        self.min_seq = max(self.min_seq, msn)  # updateSeqNumbers after the message (client.ts:1381-1391)
        self.cur_seq = seq

    # ---- f4: the local client's own events (the document's observer is that client) ----
    def local_op(self, op: dict) -> None:
        """A local submission (insertSegmentLocal / removeRangeLocal / annotateRangeLocal,
        client.ts:273-355): op contents with positions in the local view. A GROUP op (localTransaction,
        client.ts:1600-1629) submits its members one by one."""
        members = op["ops"] if op["type"] == MT_GROUP else [op]
        for m in members:
            if m["type"] not in (MT_INSERT, MT_REMOVE, MT_ANNOTATE):
                raise UnsupportedOp("local obliterate")
            self._note_op(m)
            rec = self.owner._pack(m, 0, self.cur_seq, 0, 0)
            if rec[9] & (MT_F_REL1 | MT_F_REL2):
                raise UnsupportedOp("local op with relative positions")
            self.local = True
            self.pending.append((rec[8], rec[5], self.cur_seq))
            self.ops.append(rec[:-1] + (rec[-1] | MT_F_LOCAL,))

    def local_rollback(self) -> None:
        """Rollback of the newest pending op (client.ts:554; a GROUP op: call once per member)."""
        if not self.pending:
            raise ValueError("rollback without a pending local op")
        t, payload, _ = self.pending.pop()
        self.ops.append((0, 0, 0, 0, 0, payload, 0, 0, t, MT_F_ROLLBACK))

    def local_regen(self, new_ops: list | None = None, new_client_id: str | None = None) -> None:
        """Reconnect: regeneratePendingOp for every pending op (client.ts:1452-1542). The ops it
        returns (one per segment of each pending op, in order: what fmt_mt_fetch_regen returns)
        become the pending ops, whose acks follow as the local client's messages: pass them here, or
        to regen_pending once known. new_client_id: the clientId of the new connection, which keeps
        the local client's short id 0 (startOrUpdateCollaboration, client.ts:1719-1725: the old long
        id stays mapped too), so its resubmitted ops come back as acks, not as remote ops."""
        if new_client_id is not None:
            self.rename_local(new_client_id)
        self.local = True
        self.ops.append((0, 0, 0, 0, 0, 0, 0, 0, 0, MT_F_REGEN))
        # a resubmitted op keeps its original refSeq (sequence.ts:782-790): the regenerated ops' refSeqs
        # are the old pending ops', whose oldest bounds the engine's minSeq as before
        self.regen_ref = min([p[2] for p in self.pending], default=self.cur_seq)
        self.pending = []
        if new_ops is not None:
            self.regen_pending(new_ops)

    def rename_local(self, new_client_id: str) -> None:
        """startOrUpdateCollaboration with a new long id (client.ts:1719-1725): it names short id 0
        from now on; the old one keeps mapping to 0."""
        i = self.client_ids.get(new_client_id)
        if i is not None and i != 0:
            raise UnsupportedOp("a reconnect clientId that already names another client")
        self.client_ids[new_client_id] = 0
        self.client_names[0] = new_client_id

    def regen_pending(self, new_ops: list) -> None:
        self.pending = []
        for op in new_ops:
            t = op["type"]
            payload = self.owner._props_op(op.get("props") or {}, op.get("adjust")) if t == MT_ANNOTATE else 0
            self.pending.append((t, payload, self.regen_ref))

    def add_op(self, seq, ref_seq, min_seq, client, op: dict) -> None:
        self._note_op(op)
        self.ops.append(self.owner._pack(op, seq, ref_seq, min_seq, client))
        if 0 < client < len(self.last_stamp):
            self.last_stamp[client] = max(self.last_stamp[client] or seq, seq)
        self.min_seq = max(self.min_seq, min_seq)


class MergeTreeStreamBuilder:
    """Packs many documents' sequenced merge-tree messages into one MergeTreeBatch."""

    def __init__(self, keep_messages: bool = False):
        self.keep_messages = keep_messages
        self.keys = Dictionary()
        self.values = Dictionary(["null"])
        self.text: list[np.ndarray] = []
        self.text_len = 0
        self.props_ops: dict[tuple, int] = {}
        self.props_list: list[tuple] = []
        self.docs: list[_DocBuilder] = []
        self.doc_init: list[tuple] = []
        self.snapshots: list[tuple] = []  # per doc: (first_seg, n_header, n_body, min_seq, seq, loaded)
        self.snapshot_segs: list[tuple] = []
        self.seg_doc: list[int] = []  # per snapshot segment: its document
        self.relpos: list[tuple] = []  # (marker value id, offset, flags, 0)
        self.snapshot_info: list[tuple] = []  # per snapshot segment: (ins_seq, ins_client, rm_first, rm_count)
        self.snapshot_stamps: list[tuple] = []  # (seq, client, kind, 0)
        self.has_merge_info = False
        self.adjusts: list[tuple] = []  # fmt_mt_adjust rows (delta, min, max, flags, 0)
        self.adjust_rows: dict = {}

    def _relpos(self, rp: dict) -> int:
        """An IRelativePosition {id?, before?, offset?}: its row in the relpos table. The id is looked
        up as the JSON value a marker's "markerId" property holds (an id no marker holds resolves to
        no marker: posFromRelativePos returns -1, mergeTree.ts:1462-1483)."""
        mid = rp.get("id")
        marker = self.values.intern(js_json(mid)) if mid else NO_MARKER
        self.keys.intern(MARKER_ID_KEY)
        off = rp.get("offset")
        self.relpos.append((marker, int(off) if off is not None else 0, REL_BEFORE if rp.get("before") else 0, 0))
        return len(self.relpos) - 1

    def _positions(self, op) -> tuple:
        """(pos1, pos2, flags) of a range/insert op: getValidOpRange (client.ts:758-767) takes pos1/pos2
        and falls back to relativePos1/2 only when the number is undefined."""
        flags = 0
        p1, p2 = op.get("pos1"), op.get("pos2")
        if p1 is None and op.get("relativePos1") is not None:
            p1, flags = self._relpos(op["relativePos1"]), flags | MT_F_REL1
        if p2 is None and op.get("relativePos2") is not None:
            p2, flags = self._relpos(op["relativePos2"]), flags | MT_F_REL2
        if p1 is None:
            raise ValueError("op without pos1 or relativePos1")
        return int(p1), (int(p2) if p2 is not None else None), flags

    def _text(self, s: str) -> tuple:
        u = utf16(s)
        off = self.text_len
        self.text.append(u)
        self.text_len += len(u)
        return off, len(u)

    def _unit(self, v: int) -> int:
        """One UTF-16 unit in the arena (a Marker's refType); returns its offset."""
        off = self.text_len
        self.text.append(np.array([v], dtype="<u2"))
        self.text_len += 1
        return off

    def _adjust_row(self, params) -> int:
        """An AdjustParams {delta, min?, max?} (ops.ts:191-208) as an fmt_mt_adjust row. JSON null
        delta adds 0 (number + null); a null min / max is present (!== undefined) and compares as 0."""
        if not isinstance(params, dict) or "delta" not in params:
            raise UnsupportedOp("adjust without a delta")

        def num(v):
            if v is None:
                return None
            if isinstance(v, bool) or not isinstance(v, (int, float)):
                raise UnsupportedOp("non-numeric adjust parameter")
            return float(v)

        delta = num(params["delta"])
        flags, lo, hi = 0, 0.0, 0.0
        if "min" in params:
            flags |= ADJ_MIN | (ADJ_MIN_NULL if params["min"] is None else 0)
            lo = num(params["min"]) or 0.0
        if "max" in params:
            flags |= ADJ_MAX | (ADJ_MAX_NULL if params["max"] is None else 0)
            hi = num(params["max"]) or 0.0
        row = (0.0 if delta is None else delta, lo, hi, flags, 0)
        i = self.adjust_rows.get(row)
        if i is None:
            i = len(self.adjusts)
            self.adjust_rows[row] = i
            self.adjusts.append(row)
        return i

    def _props_op(self, props: dict, adjust: dict | None = None) -> int:
        """A props op: the raw (key, value) changes in JS key order, then the adjust changes
        (segmentPropertiesManager.ts:86-95 opToChanges). Held as entries (key, value id) and
        (key, -1, adjust row) over the builder's batch-wide value dictionary; finish() packs them as
        (key << 16) | value words, each adjust as (key, FMT_MT_VALUE_ADJUST) followed by its row index,
        with batch-global or document-local value ids."""
        kv = []
        for k in js_key_order(list(props)):
            v = props[k]
            key_id = self.keys.intern(k)
            if key_id > 0xFFFF:
                raise UnsupportedOp("more than 65536 distinct property keys in a batch")
            kv.append((key_id, 0 if v is None else self.values.intern(js_json(v))))
        for k in js_key_order(list(adjust or {})):
            key_id = self.keys.intern(k)
            if key_id > 0xFFFF:
                raise UnsupportedOp("more than 65536 distinct property keys in a batch")
            kv.append((key_id, -1, self._adjust_row(adjust[k])))
        t = tuple(kv)
        i = self.props_ops.get(t)
        if i is None:
            i = len(self.props_list)
            self.props_ops[t] = i
            self.props_list.append(t)
        return i

    def _pack(self, op, seq, ref, msn, client) -> tuple:
        if op is None:  # empty group: only advances the collab window
            return (seq, ref, msn, 0, 0, 0, 0, client, MT_REMOVE, 0)
        t = op["type"]
        if t == MT_INSERT:
            p1, _, rel = self._positions({"pos1": op.get("pos1"), "relativePos1": op.get("relativePos1")})
            seg = op["seg"]
            props = None
            rtype = marker_ref_type(seg)
            if rtype is not None:  # Marker.make(refType, props): len 1, its arena unit = refType
                props = seg.get("props")
                pos2 = -1 if props is None else self._props_op(props) + 1
                return (seq, ref, msn, p1, pos2, self._unit(rtype), 1, client, MT_INSERT, MT_F_MARKER | rel)
            if not isinstance(seg, str):  # IJSONTextSegment {text, props} (textSegment.ts:44-52)
                if isinstance(seg, dict) and "text" in seg and set(seg) <= {"text", "props"}:
                    props = seg.get("props")
                    seg = seg["text"]
                else:
                    raise UnsupportedOp("segment spec")
            off, n = self._text(seg)
            if n > MAX_INSERT_UNITS:
                raise UnsupportedOp("insert longer than 2^24 - 1 UTF-16 units")
            # pos2: the segment's props-op id + 1 (TextSegment.make(text, props)); -1: a plain string
            pos2 = -1 if props is None else self._props_op(props) + 1
            # a length past 16 bits keeps its bits 16..23 in flags (FMT_MT_F_LEN_HI_SHIFT)
            return (seq, ref, msn, p1, pos2, off, n & 0xFFFF, client, MT_INSERT, rel | (n & MT_F_LEN_HI_MASK))
        if t == MT_REMOVE:
            p1, p2, rel = self._positions(op)
            return (seq, ref, msn, p1, p2, 0, 0, client, MT_REMOVE, rel)
        if t == MT_OBLITERATE:  # non-sided obliterate: {pos1, Before} .. {pos2 - 1, After}
            return (seq, ref, msn, int(op["pos1"]), int(op["pos2"]), 0, 0, client, MT_OBLITERATE, 0)
        if t == MT_OBLITERATE_SIDED:  # places {pos, before} (client.ts:680-700); sides in flags
            p1, p2 = op["pos1"], op["pos2"]
            flags = (MT_F_START_BEFORE if p1["before"] else 0) | (MT_F_END_BEFORE if p2["before"] else 0)
            return (seq, ref, msn, int(p1["pos"]), int(p2["pos"]), 0, 0, client, MT_OBLITERATE_SIDED, flags)
        if t == MT_ANNOTATE:  # IMergeTreeAnnotateMsg props and/or IMergeTreeAnnotateAdjustMsg adjust
            p1, p2, rel = self._positions(op)
            pid = self._props_op(op.get("props") or {}, op.get("adjust"))
            return (seq, ref, msn, p1, p2, pid, 0, client, MT_ANNOTATE, rel)
        raise UnsupportedOp(f"merge-tree op type {t}")

    def begin_doc(self, initial_text: str = "", observer: str = "A") -> _DocBuilder:
        d = _DocBuilder(self, observer)
        self.docs.append(d)
        self.doc_init.append(self._text(initial_text) if initial_text else (0, 0))
        self.snapshots.append((0, 0, 0, 0, 0, 0))
        return d

    def _spec(self, spec) -> tuple:
        """specToSegment: "text", {"text", "props"} (IJSONTextSegment) or a Marker spec."""
        rtype = marker_ref_type(spec)
        if rtype is not None:
            props = spec.get("props")
            return (self._unit(rtype), 1 | MT_SEG_MARKER, self._props_op(props) if props else NO_PROPS)
        if isinstance(spec, str):
            text, props = spec, None
        elif isinstance(spec, dict) and "text" in spec and set(spec) <= {"text", "props"}:
            text, props = spec["text"], spec.get("props")
        else:
            raise UnsupportedOp("markers and segments with merge info (SnapshotV1) are not loaded")
        off, n = self._text(text)
        if n == 0:
            raise ValueError("empty segment in a summary chunk")
        return (off, n, self._props_op(props) if props else NO_PROPS)

    def begin_doc_from_summary(self, header: str, body=None, catchup_ops: str | None = None,
                               observer: str = "snapshot") -> _DocBuilder:
        """A document that starts from a SharedString summary (SnapshotLoader, snapshotLoader.ts:
        59-348): the header/body chunk blobs (a legacy "body", or SnapshotV1's "body_0", "body_1", ...
        as a list, toLatestVersion snapshotChunks.ts:151-180) and, optionally, the legacy catchupOps
        blob, whose messages are added as the first ops after validation as
        SharedSegmentSequence.loadCore does (sequence.ts:818-863). The loading client is `observer`
        (short id 0). V1 header-chunk segments that carry merge info (seq/client/removed and moved
        stamps above minSeq) load with their stamps as specToSegment builds them
        (snapshotLoader.ts:105-175); body-chunk segments then load as FMT_MT_F_LOADSEG inserts (below)."""
        h = json.loads(header)
        md = h.get("headerMetadata")
        if md is None:
            raise ValueError("header metadata not available")
        bodies = [] if body is None else ([body] if isinstance(body, str) else list(body))
        chunks = [h] + [json.loads(b) for b in bodies]
        if len(md["orderedChunkMetadata"]) != len(chunks):
            raise ValueError("summary chunks do not match headerMetadata.orderedChunkMetadata")

        def specs(c):
            return c["segments"] if c.get("version") == "1" else c["segmentTexts"]

        seq = int(md["sequenceNumber"])
        min_seq = int(md.get("minSequenceNumber", seq))
        d = _DocBuilder(self, observer)
        d.min_seq = min_seq  # the loaded tree's minSeq (loadCore → MergeTree.startCollaboration)
        d.cur_seq = seq
        first = len(self.snapshot_segs)
        any_info = False
        for ci, c in enumerate(chunks):
            for spec in specs(c):
                info = (0, NON_COLLAB_CLIENT, 0, 0)
                if isinstance(spec, dict) and "json" in spec:  # hasMergeInfo
                    info = self._merge_info(spec, d)
                    spec = spec["json"]
                    any_info = True
                if marker_ref_type(spec) is not None:  # loaded markers register their ids too
                    d.note_marker_id(spec.get("props"))
                self.snapshot_segs.append(self._spec(spec))
                self.snapshot_info.append(info)
        self.seg_doc.extend([len(self.docs)] * (len(self.snapshot_segs) - first))
        n_header = len(specs(h))
        n_body = len(self.snapshot_segs) - first - n_header
        if n_header + n_body != md["totalSegmentCount"]:
            raise ValueError("Mismatch in totalSegmentCount")  # snapshotLoader.ts:272-275
        self.docs.append(d)
        self.doc_init.append((0, 0))
        if any_info and n_body:
            # loadBody with merge info (snapshotLoader.ts:254-309): each body segment is appended through
            # insertSegments at the local length from PriorPerspective(0, its client) — a batch of
            # segments without merge info in one call — so they become FMT_MT_F_LOADSEG inserts ahead of
            # the messages (their specs and merge info rows stay in the tables; the document loads its
            # header alone)
            # The reference's flushBatch (snapshotLoader.ts:291-296) never clears `batch`: once a segment
            # without merge info precedes one with merge info, every later flush inserts the batched
            # segment objects AGAIN (overwriteInfo + insertingWalk on segments already in the tree,
            # mergeTree.ts:1609-1626), aliasing them in two blocks. That state has no consistent
            # segment list to reproduce, so such a body is refused rather than loaded differently.
            universal_seen = False
            for k in range(first + n_header, first + n_header + n_body):
                ins_seq, ins_client = self.snapshot_info[k][0], self.snapshot_info[k][1]
                universal = ins_client == NON_COLLAB_CLIENT and ins_seq == 0
                if universal_seen and not universal:
                    raise UnsupportedOp("a SnapshotV1 body where a segment without merge info precedes one with "
                                        "merge info (the reference's loadBody re-inserts the batched segments)")
                universal_seen = universal_seen or universal
            prev_universal = False
            for k in range(first + n_header, first + n_header + n_body):
                off, ln, pid = self.snapshot_segs[k]
                ins_seq, ins_client = self.snapshot_info[k][0], self.snapshot_info[k][1]
                universal = ins_client == NON_COLLAB_CLIENT and ins_seq == 0
                n_units = ln & ~MT_SEG_MARKER
                flags = MT_F_LOADSEG | (MT_F_MARKER if ln & MT_SEG_MARKER else 0) | (n_units & MT_F_LEN_HI_MASK)
                if universal and prev_universal:
                    flags |= MT_F_GROUP_CONT
                prev_universal = universal
                if n_units > 0xFFFFFF:
                    raise UnsupportedOp("a SnapshotV1 body segment longer than 2^24 - 1 UTF-16 units")
                client = CLIENT_NONCOLLAB_OP if ins_client == NON_COLLAB_CLIENT else ins_client
                d.ops.append((ins_seq, 0, min_seq, k, pid + 1 if pid != NO_PROPS else 0, off, n_units & 0xFFFF, client,
                              MT_INSERT, flags))
            n_body = 0
        self.snapshots.append((first, n_header, n_body, min_seq, seq, 1))
        if catchup_ops is not None:
            cur = seq
            for m in json.loads(catchup_ops):
                if (m["minimumSequenceNumber"] < min_seq or m["referenceSequenceNumber"] < min_seq
                        or m["sequenceNumber"] <= min_seq or m["sequenceNumber"] < cur):
                    raise ValueError("Invalid catchup operations in snapshot")  # sequence.ts:838-858
                cur = m["sequenceNumber"]
                d.add_message(m)
        return d

    def _merge_info(self, spec: dict, d: _DocBuilder) -> tuple:
        """specToSegment's stamps (snapshotLoader.ts:105-175): insert {seq ?? 0, client ?? NonCollab};
        setRemove stamps at removedSeq for every removedClientIds entry (removedClient alone in the
        back-compat format), sliceRemove stamps movedSeqs[i] / movedClientIds[i], sorted by seq
        (opstampUtils.compare; Array.prototype.sort is stable)."""
        self.has_merge_info = True
        ins_seq = int(spec.get("seq", 0))
        ins_client = d.short_client(spec["client"], ins_seq) if spec.get("client") is not None else NON_COLLAB_CLIENT
        stamps = []
        if spec.get("removedSeq") is not None:
            ids = spec.get("removedClientIds")
            if ids is None and spec.get("removedClient") is not None:
                ids = [spec["removedClient"]]
            if ids is None:
                raise ValueError("must have removedClient ids")  # 0xaac
            stamps += [(int(spec["removedSeq"]), d.short_client(c, int(spec["removedSeq"])), 0) for c in ids]
        if spec.get("movedSeq") is not None:
            seqs, ids = spec.get("movedSeqs"), spec.get("movedClientIds")
            if seqs is None or ids is None or len(seqs) != len(ids):
                raise ValueError("must have movedIds ids")  # 0xaa5 / 0xb5f
            stamps += [(int(s), d.short_client(c, int(s)), 1) for s, c in zip(seqs, ids)]
        stamps.sort(key=lambda x: x[0])
        first = len(self.snapshot_stamps)
        self.snapshot_stamps += [(s, c, k, 0) for s, c, k in stamps]
        return (ins_seq, ins_client, first, len(stamps))

    def finish(self, catchup: bool = False, remove_order: bool = False) -> MergeTreeBatch:
        """The packed batch. With `catchup`, ops of messages that stay in the legacy summary's
        catch-up window get FMT_MT_F_CATCHUP (see flag_catchup); with `remove_order`, the removes
        a SnapshotV1 summary needs get FMT_MT_F_RMORDER (see flag_remove_order)."""
        n = sum(d.n_ops for d in self.docs)
        ops = np.zeros(n, dtype=MT_OP_DTYPE)
        offs = np.zeros(len(self.docs) + 1, dtype=np.uint64)
        i = 0
        for di, d in enumerate(self.docs):
            if d.ops:
                ops[i : i + d.n_ops] = np.array(d.ops, dtype=MT_OP_DTYPE)
            i += d.n_ops
            offs[di + 1] = i
        if catchup:
            flag_catchup(ops, offs)
        if remove_order:
            flag_remove_order(ops, offs)
        text = np.concatenate(self.text) if self.text else np.zeros(0, dtype="<u2")
        segs = np.array(self.snapshot_segs, dtype=SNAPSHOT_SEG_DTYPE)
        relpos = np.array(self.relpos, dtype=RELPOS_DTYPE) if self.relpos else None
        # value ids: batch-global while the batch's distinct values fit below the id limit
        # (FMT_MT_VALUE_COMPUTED with adjusts, else FMT_MT_VALUE_ADJUST), else document-local
        # (fmt.h doc_value_base): every document gets its own dictionary and props ops
        limit = VALUE_COMPUTED if self.adjusts else VALUE_ADJUST
        if len(self.values.items) <= limit:
            props_list, values, value_base = self.props_list, list(self.values.items), None
        else:
            props_list, values, value_base = self._localize_values(ops, offs, segs, relpos, limit)
        props_off = np.zeros(len(props_list) + 1, dtype=np.uint32)
        kv = []
        for j, t in enumerate(props_list):
            for e in t:
                kv += [(e[0] << 16) | e[1]] if len(e) == 2 else [(e[0] << 16) | VALUE_ADJUST, e[2]]
            props_off[j + 1] = len(kv)
        return MergeTreeBatch(
            ops=ops,
            doc_op_offsets=offs,
            text=np.ascontiguousarray(text, dtype="<u2"),
            doc_init=np.asarray(self.doc_init, dtype=np.uint32).reshape(-1, 2),
            props_off=props_off,
            props_kv=np.asarray(kv, dtype=np.uint32),
            keys=list(self.keys.items),
            values=values,
            clients=[list(d.client_names) for d in self.docs],
            messages=[list(d.messages) for d in self.docs] if self.keep_messages else [],
            snapshots=_snapshot_array(self.snapshots),
            snapshot_segs=segs,
            relpos=relpos,
            snapshot_info=np.array(self.snapshot_info, dtype=SNAPSHOT_INFO_DTYPE) if self.has_merge_info else None,
            snapshot_stamps=np.array(self.snapshot_stamps, dtype=STAMP_DTYPE) if self.has_merge_info else None,
            marker_id_key=self.keys.ids.get(MARKER_ID_KEY, NO_MARKER) if self.relpos else NO_MARKER,
            adjusts=np.array(self.adjusts, dtype=ADJUST_DTYPE) if self.adjusts else None,
            value_num=value_numbers(values) if self.adjusts else None,
            value_base=value_base,
        )

    def _localize_values(self, ops, offs, segs, relpos, limit):
        """Document-local value ids: every props op a document references (annotate payloads, insert
        props pos2 - 1, its summary segments' props) becomes a props op of that document alone whose
        values are numbered 1.. in the document's own dictionary, and its relative positions' marker
        ids follow. Rewrites ops / segs / relpos in place; returns (props ops, values, value_base)."""
        n_docs = len(offs) - 1
        doc_of = np.repeat(np.arange(n_docs, dtype=np.int64), np.diff(offs.astype(np.int64)))
        t = ops["type"]
        ann = np.nonzero(t == MT_ANNOTATE)[0]
        ins = np.nonzero((t == MT_INSERT) & (ops["pos2"] > 0))[0]
        seg_doc = np.asarray(self.seg_doc, dtype=np.int64)
        sgp = np.nonzero(segs["props"] != NO_PROPS)[0] if len(segs) else np.zeros(0, np.int64)
        n_p = max(1, len(self.props_list))
        keys = np.concatenate([doc_of[ann] * n_p + ops["payload"][ann].astype(np.int64),
                               doc_of[ins] * n_p + (ops["pos2"][ins].astype(np.int64) - 1),
                               seg_doc[sgp] * n_p + segs["props"][sgp].astype(np.int64)])
        uniq, inv = np.unique(keys, return_inverse=True)
        na, ni = len(ann), len(ins)
        ops["payload"][ann] = inv[:na].astype(np.uint32)
        ops["pos2"][ins] = (inv[na : na + ni] + 1).astype(np.int32)
        if len(sgp):
            segs["props"][sgp] = inv[na + ni :].astype(np.uint32)
        local: list[dict] = [dict() for _ in range(n_docs)]  # per document: batch value id → local id

        def lid(d, g):
            m = local[d]
            v = m.get(g)
            if v is None:
                v = m[g] = len(m) + 1
            return v

        props_list = []
        for u in uniq.tolist():
            d, pid = divmod(u, n_p)
            props_list.append(tuple((e[0], 0 if e[1] == 0 else lid(d, e[1])) if len(e) == 2 else e
                                    for e in self.props_list[pid]))
        if relpos is not None:
            for flag, field in ((MT_F_REL1, "pos1"), (MT_F_REL2, "pos2")):
                for i in np.nonzero(ops["flags"] & flag)[0].tolist():
                    row = int(ops[field][i])
                    if relpos["marker_id"][row] != NO_MARKER:
                        relpos["marker_id"][row] = lid(int(doc_of[i]), int(relpos["marker_id"][row]))
        values, base = ["null"], np.zeros(n_docs + 1, dtype=np.uint32)
        for d in range(n_docs):
            if len(local[d]) >= limit:
                raise UnsupportedOp(f"more than {limit - 1} distinct property values in one document")
            base[d] = len(values) - 1
            values += [self.values.items[g] for g in local[d]]  # (dicts keep insertion order)
        base[n_docs] = len(values) - 1
        return props_list, values, base


def _snapshot_array(rows) -> np.ndarray | None:
    if not any(r[5] for r in rows):
        return None
    a = np.zeros(len(rows), dtype=SNAPSHOT_DOC_DTYPE)
    for i, (first, nh, nb, msn, seq, loaded) in enumerate(rows):
        a[i] = (first, nh, nb, msn, seq, loaded, 0)
    return a


def flag_catchup(ops: np.ndarray, offs: np.ndarray) -> None:
    """Set FMT_MT_F_CATCHUP on the ops whose message SharedSegmentSequence keeps for the legacy
    summary's catch-up blob with regenerated contents: seq above the document's final minSeq
    (processMinSequenceNumberChanged at summarize, sequence.ts:949-963, 1008-1018) and
    refSeq != seq - 1 (needsTransformation, sequence.ts:978)."""
    offs = np.asarray(offs, dtype=np.int64)
    n = np.diff(offs)
    if not len(ops):
        return
    last = np.maximum(offs[1:] - 1, 0)
    final_msn = np.repeat(ops["min_seq"][last], n)  # each op's document's final minSeq
    sel = (ops["seq"] > final_msn) & (ops["ref_seq"] != ops["seq"] - 1) & ((ops["flags"] & MT_F_LOADSEG) == 0)
    ops["flags"][sel] |= MT_F_CATCHUP


def op_messages(batch, d: int, above_seq: int, names) -> list:
    """[(message, first op, 1)] for the ops of document d with seq > above_seq, as the
    ISequencedDocumentMessage a single-op-per-message stream (the generated farms) carries:
    {clientId, sequenceNumber, referenceSequenceNumber, minimumSequenceNumber, type, contents} with the
    op rebuilt from its record (insert text / {text, props}, remove, annotate props). The catch-up
    window of a generated document, for the legacy summary's catchupOps blob."""
    a, b = int(batch.doc_op_offsets[d]), int(batch.doc_op_offsets[d + 1])
    recs = batch.ops[a:b]
    vals = batch.doc_values(d) if hasattr(batch, "doc_values") else batch.values
    out = []
    for k in np.nonzero(recs["seq"] > above_seq)[0]:
        r = recs[int(k)]
        t = int(r["type"])
        if int(r["flags"]) & MT_F_GROUP_CONT:
            raise UnsupportedOp("GROUP messages need the original messages")
        if t == MT_INSERT:
            off, ln = int(r["payload"]), op_len(r)
            op = {"pos1": int(r["pos1"]), "seg": batch.text[off : off + ln].tobytes().decode("utf-16-le", "surrogatepass"),
                  "type": t}
        elif t == MT_ANNOTATE:
            pid = int(r["payload"])
            kv = batch.props_kv[int(batch.props_off[pid]) : int(batch.props_off[pid + 1])]
            op = {"pos1": int(r["pos1"]), "pos2": int(r["pos2"]),
                  "props": {batch.keys[int(x) >> 16]: json.loads(vals[int(x) & 0xFFFF]) for x in kv}, "type": t}
        else:
            op = {"pos1": int(r["pos1"]), "pos2": int(r["pos2"]), "type": t}
        out.append(({"clientId": names[int(r["client"])], "sequenceNumber": int(r["seq"]),
                     "referenceSequenceNumber": int(r["ref_seq"]), "minimumSequenceNumber": int(r["min_seq"]),
                     "type": "op", "contents": op}, int(k), 1))
    return out


def flag_remove_order(ops: np.ndarray, offs: np.ndarray) -> None:
    """Set FMT_MT_F_RMORDER on the REMOVE, obliterate and INSERT ops above the document's final
    minSeq: the only ones that can add a later remove stamp to a leaf that a SnapshotV1 summary lists
    with merge info (snapshotV1.ts:207-265 skips leaves removed at/below minSeq); an INSERT only
    through obliterate-on-insert (mergeTree.ts:1642-1746), so inserts are flagged in documents that
    hold obliterates."""
    for d in range(len(offs) - 1):
        a, b = int(offs[d]), int(offs[d + 1])
        if a == b:
            continue
        seg = ops[a:b]
        final_msn = int(seg["min_seq"][-1])
        t = seg["type"]
        ob = (t == MT_OBLITERATE) | (t == MT_OBLITERATE_SIDED)
        kinds = (t == MT_REMOVE) | ob | ((t == MT_INSERT) & bool(ob.any()))
        sel = (seg["seq"] > final_msn) & kinds & ((seg["flags"] & MT_F_LOADSEG) == 0)
        seg["flags"][sel] |= MT_F_RMORDER


@dataclass
class MapBatch:
    ops: np.ndarray             # MAP_OP_DTYPE
    doc_op_offsets: np.ndarray  # uint64, n_docs + 1
    key_bound: int
    keys: list                  # key id → key string
    values: list                # value id → JSON text
    local_ops: np.ndarray = None      # MAP_LOCAL_OP_DTYPE: the local client's events (fmt_map_pending_run)
    local_offsets: np.ndarray = None  # uint64, n_docs + 1

    @property
    def n_docs(self) -> int:
        return len(self.doc_op_offsets) - 1


class MapStreamBuilder:
    """Packs SharedMap messages ({"type":"set"|"delete"|"clear", ...}) per document."""

    def __init__(self):
        self.keys = Dictionary()
        self.values = Dictionary()
        self.docs: list[list[tuple]] = []
        self._last_seq: dict[int, int] = {}
        self.local: list[list[tuple]] = []     # per document, its local client's events
        self._unacked: list[list[tuple]] = []  # per document, (key, kind_value) of unacknowledged submissions

    def begin_doc(self) -> int:
        self.docs.append([])
        self.local.append([])
        self._unacked.append([])
        return len(self.docs) - 1

    def _record(self, doc: int, contents: dict):
        """(key id, kind_value) of a set / delete / clear op's contents."""
        t = contents["type"]
        if t == "clear":
            return 0, MAP_CLEAR << MAP_KIND_SHIFT
        key = self.keys.intern(contents["key"])
        if t == "delete":
            return key, MAP_DELETE << MAP_KIND_SHIFT
        if t != "set":
            raise UnsupportedOp(f"map op type {t}")
        sv = contents["value"]
        if sv.get("type") != "Plain":
            raise UnsupportedOp("legacy Shared value type")
        if "value" in sv and sv["value"] is not _MISSING:
            vid = self.values.intern(js_json(sv["value"]))
            if vid >= MAP_VALUE_UNDEFINED:
                raise UnsupportedOp("value dictionary overflow")
        else:
            vid = MAP_VALUE_UNDEFINED
        return key, (MAP_SET << MAP_KIND_SHIFT) | vid

    # ---- the document's local client (MapKernel pendingData, mapKernel.ts:132-139, 388-538, 633-853)
    def local_submit(self, doc: int, contents: dict) -> None:
        """MapKernel.set / delete / clear on the attached map: the op enters pendingData (it is not
        sequenced until local_ack)."""
        key, kv = self._record(doc, contents)
        self.local[doc].append((doc, key, MAP_EV_SUBMIT, kv))
        self._unacked[doc].append((key, kv))

    def local_ack(self, doc: int, seq: int) -> None:
        """The oldest unacknowledged local op comes back sequenced: it is appended to the document's
        sequenced stream like any message and leaves pendingData (the handlers' local branches)."""
        if not self._unacked[doc]:
            raise ValueError("local_ack with no unacknowledged local op")
        key, kv = self._unacked[doc].pop(0)
        ops = self.docs[doc]
        last = self._last_seq.get(doc, 0)
        if seq < last:
            raise ValueError(f"map message seq {seq} after {last}: messages must arrive in seq order")
        self._last_seq[doc] = seq
        ops.append((doc, key, len(ops) + 1, kv))
        self.local[doc].append((doc, key, MAP_EV_ACK, kv))

    def local_rollback(self, doc: int) -> None:
        """MapKernel.rollback of the newest unacknowledged local op (mapKernel.ts:633-700)."""
        if not self._unacked[doc]:
            raise ValueError("local_rollback with no unacknowledged local op")
        key, kv = self._unacked[doc].pop()
        self.local[doc].append((doc, key, MAP_EV_ROLLBACK, kv))

    def add_message(self, doc: int, seq: int, contents: dict) -> None:
        """One sequenced map message. Messages of one runtime bunch share their envelope's
        sequenceNumber (sharedObject.ts:620-630, sequence.ts:882-888), so the record's `seq` field
        carries the message's 1-based ordinal in the document's stream instead: strictly increasing,
        it keeps a bunch's order for LWW and for JS Map insertion order (mapKernel.ts:708-850)."""
        ops = self.docs[doc]
        last = self._last_seq.get(doc, 0)
        if seq < last:
            raise ValueError(f"map message seq {seq} after {last}: messages must arrive in seq order")
        self._last_seq[doc] = seq
        seq = len(ops) + 1
        t = contents["type"]
        if t == "clear":
            ops.append((doc, 0, seq, MAP_CLEAR << MAP_KIND_SHIFT))
            return
        key = self.keys.intern(contents["key"])
        if t == "delete":
            self.docs[doc].append((doc, key, seq, (MAP_DELETE << MAP_KIND_SHIFT)))
        elif t == "set":
            sv = contents["value"]
            if sv.get("type") != "Plain":
                raise UnsupportedOp("legacy Shared value type")
            if "value" in sv and sv["value"] is not _MISSING:
                vid = self.values.intern(js_json(sv["value"]))
                if vid >= MAP_VALUE_UNDEFINED:
                    raise UnsupportedOp("value dictionary overflow")
            else:
                vid = MAP_VALUE_UNDEFINED
            self.docs[doc].append((doc, key, seq, (MAP_SET << MAP_KIND_SHIFT) | vid))
        else:
            raise UnsupportedOp(f"map op type {t}")

    def begin_doc_from_summary(self, header: str, blobs=()) -> int:
        """A document whose map starts from a SharedMap summary (SharedMap.loadCore, map.ts:251-267):
        the header's "content" entries, then each blob's, enter sequencedData in Object.entries
        order (MapKernel.populateFromSerializable, mapKernel.ts:557-564). They are packed as the
        document's first set records, so later messages apply on top in order."""
        doc = self.begin_doc()
        h = json.loads(header)
        parts = [h["content"]] + [json.loads(b) for b in blobs] if isinstance(h.get("blobs"), list) else [h]
        for part in parts:
            for key in js_key_order(list(part)):
                ser = part[key]
                value = {"type": ser.get("type", "Plain")}
                if "value" in ser:
                    value["value"] = ser["value"]
                self.add_message(doc, 0, {"type": "set", "key": key, "value": value})
        return doc

    def finish(self) -> MapBatch:
        n = sum(len(d) for d in self.docs)
        ops = np.zeros(n, dtype=MAP_OP_DTYPE)
        offs = np.zeros(len(self.docs) + 1, dtype=np.uint64)
        i = 0
        for di, d in enumerate(self.docs):
            if d:
                ops[i : i + len(d)] = np.array(d, dtype=MAP_OP_DTYPE)
            i += len(d)
            offs[di + 1] = i
        lo, loff = None, None
        if any(self.local):
            ev = [e for d in self.local for e in d]
            lo = np.array(ev, dtype=MAP_LOCAL_OP_DTYPE) if ev else np.zeros(0, dtype=MAP_LOCAL_OP_DTYPE)
            loff = np.zeros(len(self.docs) + 1, dtype=np.uint64)
            loff[1:] = np.cumsum([len(d) for d in self.local])
        return MapBatch(ops, offs, max(1, len(self.keys.items)), list(self.keys.items), list(self.values.items),
                        lo, loff)


class _Missing:
    pass


_MISSING = _Missing()
