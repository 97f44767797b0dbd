/*
 * fmt.h — C ABI of the MI355X batch merge engine ("fmt" = Fluid merge tree).
 *
 * The engine replays already-sequenced op streams for very many independent documents and
 * produces their converged DDS state. It is the drop-in for the data-parallel hot path that the
 * reference runs one message at a time through
 *
 *   SharedObjectCore.processMessagesCore            packages/dds/shared-object-base/src/sharedObject.ts:415
 *     SharedMap.processMessagesCore                 packages/dds/map/src/map.ts:288-311
 *       MapKernel.tryProcessMessage                 packages/dds/map/src/mapKernel.ts:619-630
 *     SharedSegmentSequence.processMessagesCore     packages/dds/sequence/src/sequence.ts:873-919
 *       Client.applyMsg                             packages/dds/merge-tree/src/client.ts:1358-1379
 *   summarizeCore                                   map.ts:176-246, sequence.ts:713-728
 *
 * Conventions (all entry points):
 *   - return 0 (FMT_OK) on success, a negative FMT_E_* code on failure; fmt_last_error() explains.
 *   - FMT_E_DATA is the DataProcessingError analogue (bad remote data, mergeTree.ts:1629-1638),
 *     FMT_E_USAGE the UsageError analogue (API misuse). Per-document failures are also reported in
 *     that document's result status word; the first failing (doc, seq) is recorded in the context.
 *   - Inputs are caller-owned and only read during the call. Device state is library-owned until
 *     fmt_close(). No exception ever crosses this ABI. One context per host thread.
 *   - Positions and lengths are UTF-16 code units (textSegment.ts:60), exactly like JS strings.
 */
#ifndef FMT_H_
#define FMT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------------------------------------
 * Status codes
 * ------------------------------------------------------------------------------------------- */
#define FMT_OK 0
#define FMT_E_USAGE (-1)       /* misuse: bad argument, wrong call order (UsageError analogue) */
#define FMT_E_DATA (-2)        /* invalid op stream (DataProcessingError analogue) */
#define FMT_E_CAPACITY (-3)    /* a document exceeded a per-document engine capacity */
#define FMT_E_DEVICE (-4)      /* HIP runtime failure, or no usable gfx950 device */
#define FMT_E_UNSUPPORTED (-5) /* op kind this engine build does not implement (e.g. obliterate) */

/* ---------------------------------------------------------------------------------------------
 * Constants mirrored from the reference
 * ------------------------------------------------------------------------------------------- */
/* MergeTreeDeltaType, packages/dds/merge-tree/src/ops.ts:61-71 */
#define FMT_MT_INSERT 0
#define FMT_MT_REMOVE 1
#define FMT_MT_ANNOTATE 2
#define FMT_MT_GROUP 3 /* never appears in a packed stream: group members are flattened, same seq */
#define FMT_MT_OBLITERATE 4
#define FMT_MT_OBLITERATE_SIDED 5

/* stamps.ts / constants.ts:14-42 */
#define FMT_UNIVERSAL_SEQ 0
#define FMT_LOCAL_CLIENT (-1)
#define FMT_NON_COLLAB_CLIENT (-2)
#define FMT_NOT_REMOVED 0x7fffffff

/* Map op kinds (mapKernel.ts:706-853 handlers "set" / "delete" / "clear") */
#define FMT_MAP_SET 0u
#define FMT_MAP_DELETE 1u
#define FMT_MAP_CLEAR 2u
#define FMT_MAP_KIND_SHIFT 30
#define FMT_MAP_VALUE_MASK 0x3fffffffu
#define FMT_MAP_VALUE_UNDEFINED 0x3fffffffu /* map.set(key, undefined): summary omits "value" */
#define FMT_MAP_ABSENT 0xffffffffu          /* result slot: key not live */

/* ---------------------------------------------------------------------------------------------
 * Packed op records (host driver output, the bytes that cross host→HBM once per batch)
 * ------------------------------------------------------------------------------------------- */

/* One sequenced merge-tree message (ISequencedDocumentMessage, driver-definitions protocol.ts:217,
 * with contents IMergeTreeInsertMsg / IMergeTreeRemoveMsg / IMergeTreeAnnotateMsg, ops.ts:112-235).
 * A GROUP message is flattened into consecutive records; every member after the first carries
 * FMT_MT_F_GROUP_CONT and the collab window advances once after the last member
 * (client.ts:1311-1319, 1358-1379). Separate messages that share a seq (a runtime "bunch") are NOT
 * flagged: each advances the window, exactly as each applyMsg call does. 32 bytes. */
#define FMT_MT_F_GROUP_CONT 1u
/* Record the op's regenerated "catch-up" contents: the ranges of the sequenceDelta event it raises,
 * merged as SharedSegmentSequence.createOpsFromDelta merges them (sequence/src/sequence.ts:395-452).
 * The host sets it on the ops of messages that stay in the legacy summary's catch-up window
 * (seq > final minSeq) and need transformation (refSeq != seq - 1, sequence.ts:971-1006). */
#define FMT_MT_F_CATCHUP 2u
/* Record the remove order (SnapshotV1 merge info, merge-tree/src/snapshotV1.ts:207-265): for every
 * leaf this REMOVE or obliterate hits that is already removed, append (leaf, client, seq, kind) to
 * the document's remove-order slab, so the summary can list removedClientIds and movedSeqs /
 * movedClientIds in stamp order (stamps.ts:144-158); on an INSERT, the second and later stamps an
 * obliterate-on-insert gives the new leaf (mergeTree.ts:1642-1746). The host sets it on the REMOVE,
 * obliterate and INSERT ops with seq > the document's final minSeq (only leaves removed above minSeq
 * carry merge info). The first stamp is the op whose seq is the leaf's rm_seq. */
#define FMT_MT_F_RMORDER 4u
/* FMT_MT_OBLITERATE_SIDED (mergeTreeEnableSidedObliterate, client.ts:680-700): pos1/pos2 hold
 * start.pos / end.pos of the InteriorSequencePlaces and these bits their sides (set = Side.Before,
 * clear = Side.After). A non-sided FMT_MT_OBLITERATE (pos1, pos2) is the sided {pos1, Before} ..
 * {pos2 - 1, After} (mergeTree.ts:2282-2286). */
#define FMT_MT_F_START_BEFORE 8u
#define FMT_MT_F_END_BEFORE 16u
/* INSERT of a Marker segment (seg {"marker": {"refType"}, "props"?}, mergeTreeNodes.ts:495-564):
 * cachedLength 1, never appended to or onto (canAppend false); len = 1 and the one arena unit at
 * payload holds its refType (ReferenceType bit flags). */
#define FMT_MT_F_MARKER 32u
/* Legacy relative positions (ops.ts:115-117, IRelativePosition): the op's pos1 (REL1) / pos2 (REL2)
 * was undefined and its relativePos1 / relativePos2 names a marker; the field then holds an index
 * into fmt_mt_batch.relpos. Resolved in the op's perspective as posFromRelativePos does
 * (mergeTree.ts:1462-1483, via client.ts:760-767 getValidOpRange). */
#define FMT_MT_F_REL1 64u
#define FMT_MT_F_REL2 128u
/* A SnapshotV1 body-chunk segment the loader appends (snapshotLoader.ts:254-309), an INSERT placed
 * before the document's messages: insertSegments at the local length (root.cachedLength; the op's
 * pos1 is ignored for it) from PriorPerspective(UniversalSequenceNumber, client) with stamp {seq,
 * client}, the segment's remove stamps (fmt_mt_snapshot_info row pos1 of the batch) kept, and no
 * collab-window update. client FMT_MT_CLIENT_NONCOLLAB: NonCollabClient (a segment without merge
 * info). With FMT_MT_F_GROUP_CONT it continues the previous one's insertSegments call (a batch of
 * segments without merge info): no interval boundary is made at its position. */
#define FMT_MT_F_LOADSEG 256u
#define FMT_MT_CLIENT_NONCOLLAB 0xFEu
/* INSERT longer than 65535 UTF-16 units (a large paste): flags bits 16..23 hold bits 16..23 of the
 * length, `len` its low 16 bits (inserts up to 2^24 - 1 units; fmt_mt_op_len). */
/* f4 — the local client (a Client whose own ops apply before they are sequenced). A document with
 * these records is replayed from the perspective of its own client, short client id 0 (it never
 * appears as a remote client of that document). Each flag below makes the record a local event
 * instead of a remote message:
 * FMT_MT_F_LOCAL: a submission (insertSegmentLocal / removeRangeLocal / annotateRangeLocal,
 *   client.ts:273-355): INSERT / REMOVE / ANNOTATE with positions in the local view
 *   (LocalDefaultPerspective, perspective.ts:174-184), stamped {UnassignedSequenceNumber, 0,
 *   localSeq = ++localSeq}; its segments form a pending segment group (mergeTree.ts:1410-1447). No
 *   collab-window update, no zamboni; seq / min_seq are not read. ref_seq: the refSeq the op was
 *   submitted at (SharedSegmentSequence.inFlightRefSeqs, sequence.ts:468-499, 666): while the op is
 *   pending, every collab-window update of the document takes min(message minSeq, the oldest
 *   pending op's ref_seq) (getMinInFlightRefSeq, client.ts:1374-1378); a regenerated op keeps the
 *   original's (sequence.ts:782-790). An invalid range is FMT_E_USAGE (client.ts:797-810).
 * FMT_MT_F_ACK: a sequenced message of the local client (client.ts:1367-1368 ackPendingSegment →
 *   mergeTree.ts:1325-1408 ackOp): acknowledges the OLDEST pending group with {seq, 0}; type (and an
 *   ANNOTATE's props op, whose keys PropertiesManager.ack shifts, segmentPropertiesManager.ts:248-267)
 *   must be the group's, else FMT_E_DATA; then the collab window advances like any message (a
 *   GROUP message: one ACK per member, FMT_MT_F_GROUP_CONT).
 * FMT_MT_F_ROLLBACK: rollback of the NEWEST pending group (client.ts:554 → mergeTree.ts:2388-2514;
 *   a GROUP op's members newest first); type must match.
 * FMT_MT_F_REGEN: reconnect — regeneratePendingOp for every pending group in order
 *   (client.ts:1452-1542, squash false): segments normalized (mergeTree.ts:2734-2766), then one new
 *   op per segment at its position in LocalReconnectingPerspective(currentSeq, 0, localSeq)
 *   (resetPendingDeltaToOps, client.ts:1160-1289); the new ops replace the pending groups and are
 *   returned by fmt_mt_fetch_regen. */
#define FMT_MT_F_LOCAL 512u
#define FMT_MT_F_ACK 1024u
#define FMT_MT_F_ROLLBACK 2048u
#define FMT_MT_F_REGEN 4096u
#define FMT_MT_F_LOCAL_ANY (FMT_MT_F_LOCAL | FMT_MT_F_ACK | FMT_MT_F_ROLLBACK | FMT_MT_F_REGEN)
/* fmt_mt_leaf.ins_seq / rm_seq of a stamp still pending its ack: this | its localSeq (stamps.ts:47;
 * above every sequence number, below FMT_NOT_REMOVED). Sequence numbers stay below it. */
#define FMT_MT_LOCAL_SEQ_BASE 0x40000000
#define FMT_MT_F_LEN_HI_SHIFT 16
#define FMT_MT_F_LEN_HI_MASK 0x00FF0000u
typedef struct fmt_mt_op {
  int32_t seq;      /* sequenceNumber */
  int32_t ref_seq;  /* referenceSequenceNumber */
  int32_t min_seq;  /* minimumSequenceNumber */
  int32_t pos1;     /* op.pos1 */
  int32_t pos2;     /* op.pos2; INSERT: props-op id + 1 of a {text, props} segment, <= 0 for a string */
  uint32_t payload; /* INSERT: offset of the text in the UTF-16 arena; ANNOTATE: props-op id */
  uint16_t len;     /* INSERT: text length in UTF-16 units (> 0), low 16 bits (FMT_MT_F_LEN_HI_SHIFT) */
  uint8_t client;   /* short client id (client.ts:831-855): 1..253 in order of first appearance; ids
                       64..253 are kept by the huge tier only (the others grow such a document) */
  uint8_t type;     /* FMT_MT_* */
  uint32_t flags;   /* FMT_MT_F_* */
} fmt_mt_op;
/* The full length of an INSERT record (len plus the FMT_MT_F_LEN_HI bits). */
static inline uint32_t fmt_mt_op_len(const fmt_mt_op* op) {
  return (uint32_t)op->len | (op->flags & FMT_MT_F_LEN_HI_MASK);
}

/* An IRelativePosition {id, before, offset}: `marker_id` is the value id (props_kv dictionary) of the
 * marker's id string, i.e. the value its "markerId" property holds (FMT_MT_NO_MARKER when the
 * position names none); the position is the marker's start in the op's perspective, minus
 * `offset` when `before`, else plus the marker's length (1) and `offset`. 16 bytes. */
#define FMT_MT_NO_MARKER 0xffffffffu
#define FMT_MT_REL_BEFORE 1u
typedef struct fmt_mt_relpos {
  uint32_t marker_id;
  int32_t offset; /* 0 when the position has none */
  uint32_t flags; /* FMT_MT_REL_BEFORE */
  uint32_t pad;
} fmt_mt_relpos;

/* One SharedMap message: {"type":"set","key","value"} / "delete" / "clear"
 * (map/src/internalInterfaces.ts). 16 bytes. key = per-doc key id (< key_bound); value = id of the
 * value's serialized JSON text in the host dictionary. */
typedef struct fmt_map_op {
  uint32_t doc;
  uint32_t key;
  uint32_t seq;        /* order key, strictly increasing within the document: the host packers store
                          the message's 1-based ordinal in the document's stream, because messages of
                          one runtime bunch share their envelope's sequenceNumber
                          (shared-object-base/src/sharedObject.ts:620-630) */
  uint32_t kind_value; /* (kind << 30) | value id */
} fmt_map_op;

/* A document that starts from a loaded legacy SharedString summary instead of an empty tree
 * (SnapshotLoader, merge-tree/src/snapshotLoader.ts:59-348): the header chunk's segments rebuild
 * the tree 7 per block (reloadFromSegments, mergeTree.ts:751-800), collaboration starts at
 * (min_seq, seq) from the header metadata, and the body chunk's segments are appended through the
 * inserting walk with stamp {UniversalSequenceNumber, NonCollabClient} (snapshotLoader.ts:221-311).
 * Catch-up messages follow as ordinary ops. 32 bytes. */
typedef struct fmt_mt_snapshot_doc {
  uint64_t first_seg; /* index of the document's first fmt_mt_snapshot_seg */
  uint32_t n_header;  /* segments of the header chunk */
  uint32_t n_body;    /* segments of the body chunk(s), appended after loading the header */
  int32_t min_seq;    /* headerMetadata.minSequenceNumber ?? sequenceNumber */
  int32_t seq;        /* headerMetadata.sequenceNumber */
  uint32_t loaded;    /* 0: this document does not start from a snapshot (doc_init applies) */
  uint32_t pad;
} fmt_mt_snapshot_doc;

#define FMT_MT_NO_PROPS 0xffffffffu
/* fmt_mt_snapshot_seg.len flag: the spec is a Marker ({"marker": {"refType"}, "props"?}); its one
 * arena unit holds the refType. */
#define FMT_MT_SEG_MARKER 0x80000000u
/* One segment spec of a summary chunk ("text" or {"text","props"}, IJSONTextSegment). 12 bytes. */
typedef struct fmt_mt_snapshot_seg {
  uint32_t text;  /* offset of the text in the UTF-16 arena */
  uint32_t len;   /* UTF-16 units (> 0) */
  uint32_t props; /* props-op id whose (key, value) pairs are the segment's properties, or FMT_MT_NO_PROPS */
} fmt_mt_snapshot_seg;

/* SnapshotV1 merge info of a loaded segment (IJSONSegmentWithMergeInfo, snapshotLoader.ts:105-175
 * specToSegment), parallel to fmt_mt_snapshot_seg: its insert stamp (seq 0 and client
 * FMT_NON_COLLAB_CLIENT for a segment without merge info) and its remove stamps
 * snapshot_stamps[rm_first .. rm_first + rm_count) in stamp order. 16 bytes. Header-chunk segments
 * only (reloadFromSegments places them as they are). */
typedef struct fmt_mt_snapshot_info {
  int32_t ins_seq;
  int32_t ins_client; /* short client id, or FMT_NON_COLLAB_CLIENT */
  uint32_t rm_first;
  uint32_t rm_count;
} fmt_mt_snapshot_info;
/* One remove stamp of a loaded segment: setRemove stamps carry the spec's removedSeq for every
 * removedClientIds entry, sliceRemove stamps movedSeqs[i] / movedClientIds[i]. 16 bytes. */
typedef struct fmt_mt_stamp {
  int32_t seq;
  int32_t client;
  uint32_t kind; /* FMT_MT_RM_SET / FMT_MT_RM_SLICE */
  uint32_t pad;
} fmt_mt_stamp;

/* Annotate-adjust (IMergeTreeAnnotateAdjustMsg.adjust, merge-tree/src/ops.ts:187-222): in props_kv an
 * entry (key_id << 16) | FMT_MT_VALUE_ADJUST is followed by one word, the index of its fmt_mt_adjust
 * row. The change folds into the key's current value as computePropertyValue does
 * (segmentPropertiesManager.ts:54-78), in IEEE double: (current is a number ? current : 0) + delta,
 * then max (if present) clamps, else min. A computed number gets a value id: the host dictionary's id
 * of an equal number when there is one (matchProperties compares with ===, properties.ts:32-61),
 * else FMT_MT_VALUE_COMPUTED + its index in the document's number table (fmt_mt_fetch_numbers),
 * first-computed order, one entry per distinct number. Batches with adjusts therefore keep host
 * value ids below FMT_MT_VALUE_COMPUTED. A null min / max (JSON null, !== undefined) compares as 0
 * and yields null: the key is deleted (segmentPropertiesManager.ts:112-115). 32 bytes. */
#define FMT_MT_VALUE_ADJUST 0xffffu
#define FMT_MT_VALUE_COMPUTED 0x8000u
#define FMT_MT_ADJ_MIN 1u      /* min present */
#define FMT_MT_ADJ_MIN_NULL 2u /* min present and null */
#define FMT_MT_ADJ_MAX 4u
#define FMT_MT_ADJ_MAX_NULL 8u
typedef struct fmt_mt_adjust {
  double delta; /* AdjustParams.delta (a JSON null delta adds 0) */
  double min;
  double max;
  uint32_t flags; /* FMT_MT_ADJ_* */
  uint32_t pad;
} fmt_mt_adjust;

/* A batch of merge-tree documents. Pointers are HOST pointers for fmt_mt_load(). */
typedef struct fmt_mt_batch {
  const fmt_mt_op* ops;           /* all ops, documents contiguous and in seq order */
  uint64_t n_ops;
  const uint64_t* doc_op_offsets; /* n_docs + 1 entries */
  uint32_t n_docs;
  const uint16_t* text;           /* UTF-16 arena for insert payloads and initial texts */
  uint64_t text_len;
  const uint32_t* doc_init;       /* optional: per doc (offset, len) of the initial text inserted
                                     before collaboration starts (client.replay.spec.ts:30-33), or NULL */
  const uint32_t* props_off;      /* annotate props-op table: n_props_ops + 1 offsets into props_kv */
  uint32_t n_props_ops;
  const uint32_t* props_kv;       /* (key_id << 16) | value_id; value_id 0 = null (delete key) */
  const fmt_mt_snapshot_doc* snapshots;   /* optional: n_docs entries, or NULL (f3: load from summary) */
  const fmt_mt_snapshot_seg* snapshot_segs;
  uint64_t n_snapshot_segs;
  const fmt_mt_relpos* relpos;    /* optional: the relative positions FMT_MT_F_REL1/REL2 ops index, or NULL */
  uint32_t n_relpos;
  uint32_t marker_id_key;         /* key id of "markerId" (reservedMarkerIdKey), FMT_MT_NO_MARKER if none */
  const fmt_mt_snapshot_info* snapshot_info; /* optional: n_snapshot_segs entries (V1 merge info), or NULL */
  const fmt_mt_stamp* snapshot_stamps;
  uint64_t n_snapshot_stamps;
  const fmt_mt_adjust* adjusts;   /* optional: the rows FMT_MT_VALUE_ADJUST entries index, or NULL */
  uint32_t n_adjusts;
  uint32_t n_values;              /* entries of value_num */
  const double* value_num;        /* with adjusts: per value id, the number its JSON text parses to, NaN
                                     for a non-number (typeof !== "number") */
  const uint32_t* doc_value_base; /* optional: n_docs + 1 entries, or NULL. Non-NULL: value ids are
                                     document-local — value id v >= 1 of document d's props ops and
                                     relative positions names the batch's value v + doc_value_base[d]
                                     (value_num, fmt_mt_summarize_legacy's values), and
                                     v <= doc_value_base[d + 1] - doc_value_base[d]. A batch then holds
                                     any number of distinct values, each document below the id limits
                                     (FMT_MT_VALUE_COMPUTED with adjusts, else FMT_MT_VALUE_ADJUST). NULL:
                                     value ids are batch-global. Id 0 is null either way. */
} fmt_mt_batch;

/* ---------------------------------------------------------------------------------------------
 * Results
 * ------------------------------------------------------------------------------------------- */

/* One merge-tree leaf (segment) of the converged tree, in document order, tombstones included. */
typedef struct fmt_mt_leaf {
  int32_t ins_seq;     /* insert stamp seq */
  int32_t rm_seq;      /* first (lowest) remove stamp seq, FMT_NOT_REMOVED if not removed */
  uint64_t rm_clients; /* set of short client ids 0..63 holding a remove stamp on this leaf (ids
                          64..127: fmt_mt_fetch_rm_clients_hi, 128..253: fmt_mt_fetch_rm_clients_hi2) */
  uint32_t char_off;   /* offset of this leaf's text in the document's char output */
  uint32_t len;        /* cachedLength (UTF-16 units) */
  int16_t ins_client;  /* insert stamp client */
  uint16_t props;      /* document-local prop-set id, 0xffff = properties undefined */
  uint16_t block;      /* index of the leaf's parent block in document order of leaf blocks */
  uint16_t pad;        /* FMT_MT_LEAF_MARKER | block ordinal bits 16..30 (documents beyond 65535 leaf blocks) */
} fmt_mt_leaf;
/* fmt_mt_leaf.pad flag: the leaf is a Marker (its one char unit is its refType). */
#define FMT_MT_LEAF_MARKER 0x8000u

/* Per-document result header. */
typedef struct fmt_mt_doc_result {
  int32_t status;      /* FMT_OK or FMT_E_* */
  int32_t fail_seq;    /* seq of the op that failed, when status != FMT_OK */
  int32_t cur_seq;     /* collabWindow.currentSeq */
  int32_t min_seq;     /* collabWindow.minSeq */
  uint32_t n_leaves;
  uint32_t n_chars;    /* total chars of all leaves (tombstones included) */
  uint32_t n_props;    /* number of document-local prop sets */
  uint32_t n_blocks;   /* number of leaf blocks */
  uint32_t depth;      /* tree depth (1 = root holds leaves) */
  uint32_t visible_len;/* getLength() from the local perspective */
  uint32_t n_catchup;  /* catch-up ranges recorded for FMT_MT_F_CATCHUP ops (fmt_mt_fetch_catchup) */
  uint32_t n_rm_order; /* remove-order entries recorded for FMT_MT_F_RMORDER ops (fmt_mt_fetch_remove_order) */
} fmt_mt_doc_result;

/* One regenerated catch-up op range (a merged ISequenceDeltaRange, sequence.ts:395-452): positions
 * are in the local view right after the op applied, before its zamboni pass
 * (mergeTree.ts:1503-1516, 2069-2080, 2364-2382; SequenceDeltaEventClass positions via
 * Client.getPosition, sequenceDeltaEvent.ts:91-103). INSERT: [pos1, pos1 + text length);
 * REMOVE: newly removed segments, merged while they start at the same position; ANNOTATE:
 * annotated segments not removed, merged while contiguous. Ranges of one op are in document order. */
typedef struct fmt_mt_catchup_range {
  uint32_t op;   /* index of the op record within its document (0 = doc_op_offsets[d]) */
  int32_t pos1;
  int32_t pos2;
  uint32_t type; /* FMT_MT_INSERT / FMT_MT_REMOVE / FMT_MT_ANNOTATE */
} fmt_mt_catchup_range;

/* One later remove stamp of a leaf (the second, third, ... of its stamps.ts remove list; the first
 * is the leaf's rm_seq): `leaf` is the index in the document's final leaf list, or FMT_MT_LEAF_GONE
 * when that leaf was dropped by zamboni before the end. A split leaf's entries are copied to its
 * right part. The entries of one leaf sorted by seq follow the stamp order. 16 bytes. */
#define FMT_MT_LEAF_GONE 0xffffffffu
#define FMT_MT_RM_SET 0u   /* "setRemove": a REMOVE op (markRangeRemoved) */
#define FMT_MT_RM_SLICE 1u /* "sliceRemove": an obliterate, incl. obliterate-on-insert (mergeTree.ts:2270) */
typedef struct fmt_mt_remove_order {
  uint32_t leaf;
  int32_t client; /* short client id of the remove stamp */
  int32_t seq;    /* the stamp's seq (SnapshotV1 movedSeqs) */
  uint32_t kind;  /* FMT_MT_RM_SET / FMT_MT_RM_SLICE */
} fmt_mt_remove_order;

/* A document-local prop set: n (key_id, value_id) pairs in JS insertion order, n <=
 * FMT_MT_PROPS_KEYS_MAX. A record holds FMT_MT_PROPS_MAX of them; a set with more takes
 * ceil(n / FMT_MT_PROPS_MAX) consecutive records: the first holds n and entries 0..7, each following
 * one n = FMT_MT_PROPS_CONT and the next 8 entries (unused entries 0). Leaf prop-set ids name first
 * records; fmt_mt_doc_result.n_props counts records. */
#define FMT_MT_PROPS_MAX 8
#define FMT_MT_PROPS_KEYS_MAX 128
#define FMT_MT_PROPS_CONT 0xffffffffu
typedef struct fmt_mt_propset {
  uint32_t n;
  uint32_t kv[FMT_MT_PROPS_MAX]; /* (key_id << 16) | value_id */
} fmt_mt_propset;

/* One SharedMap result slot (per doc, per key id < key_bound). */
typedef struct fmt_map_slot {
  uint32_t value;     /* value id, FMT_MAP_VALUE_UNDEFINED, or FMT_MAP_ABSENT (not live) */
  uint32_t birth_seq; /* order key (fmt_map_op.seq) of the set that created the live entry: JS Map
                         insertion order */
} fmt_map_slot;

/* Run statistics of the last fmt_*_run (device time measured with HIP events on the ctx stream). */
typedef struct fmt_stats {
  double kernel_ms;      /* replay kernel(s) only */
  double total_ms;       /* everything launched by the run call */
  uint64_t ops;          /* messages applied */
  uint64_t docs;
  uint64_t bytes_read;   /* algorithmic bytes read by the replay kernel */
  uint64_t bytes_written;/* algorithmic bytes written by the replay kernel */
  uint64_t launches;     /* kernel launches issued by the run call */
} fmt_stats;

/* ---------------------------------------------------------------------------------------------
 * Context
 * ------------------------------------------------------------------------------------------- */
typedef struct fmt_ctx fmt_ctx;

typedef struct fmt_config {
  int32_t device;      /* HIP device ordinal */
  uint32_t flags;      /* reserved, 0 */
  void* stream;        /* hipStream_t to launch on (e.g. torch's current stream); NULL = own stream */
  uint32_t reserved[4];
} fmt_config;

/* Context lifetime. Replaces the per-DDS state owned by each SharedMap / SharedString instance
 * (map/src/map.ts:66 MapKernel construction; sequence/src/sequence.ts:526 Client construction): one ctx holds the replay state of many documents on one device. */
int fmt_open(const fmt_config* cfg, fmt_ctx** out);
void fmt_close(fmt_ctx* ctx);
/* Message of the last failing call. Replaces the thrown DataProcessingError / UsageError text
 * (merge-tree/src/mergeTree.ts:1629-1638; core-utils assert 0xNNN codes). */
const char* fmt_last_error(const fmt_ctx* ctx);
/* Wait for the ctx stream. The reference is synchronous and non-reentrant (sequence.ts:500-511). Map runs
 * are asynchronous until fmt_sync or a fetch; fmt_mt_run returns once the replay is done (it reads
 * the overflow count on the host to size the large-tier launch). */
int fmt_sync(fmt_ctx* ctx);
/* Device time and algorithmic bytes of the last run (no reference counterpart; telemetry only). */
int fmt_get_stats(const fmt_ctx* ctx, fmt_stats* out);
/* Name of the gfx target the library was built for and the device it runs on (diagnostics). */
int fmt_device_info(fmt_ctx* ctx, char* buf, size_t cap);

/* Bulk legacy SharedString summaries of every document of the last fmt_mt_run (replaces
 * SharedString.summarizeCore → SnapshotLegacy.extractSync + emit, snapshotlegacy.ts:74-262 and
 * snapshotChunks.ts:85-204, for all documents at once; catch-up ops are not included): the segment
 * merge runs on the device (one wave per document), the JSON on `threads` host threads (0 = up to
 * 16). keys: the batch's key strings JSON-quoted; values: the value JSON texts (UTF-8). Computed
 * annotate-adjust numbers are written as JSON.stringify writes them. Segment properties are
 * getAtSeq(properties, minSeq) (snapshotlegacy.ts:211-212): in batches with annotate-adjust the engine
 * keeps every segment's PropertiesManager (msnConsensus and pending remote changes,
 * segmentPropertiesManager.ts:140-345) and evaluates it at the end of the replay
 * (fmt_mt_fetch_legacy_props). */
typedef struct fmt_summary_timing {
  double kernel_ms;   /* device merge (events) */
  double fetch_ms;    /* device -> host of runs, text and prop sets */
  double format_ms;   /* host JSON */
  uint64_t bytes;     /* blob bytes produced */
  uint32_t threads;
  uint32_t pad;
} fmt_summary_timing;
int fmt_mt_summarize_legacy(fmt_ctx* ctx, const char* const* keys, uint32_t n_keys, const char* const* values,
                            uint32_t n_values, uint32_t chunk_size, uint32_t threads, fmt_summary_timing* timing);
/* Document d's blobs from the last fmt_mt_summarize_legacy (valid until the next one): header and
 * body (body_len 0: no body chunk). The replay's status when the document failed. */
int fmt_mt_summary_blobs(fmt_ctx* ctx, uint32_t doc, const char** header, size_t* header_len, const char** body,
                         size_t* body_len);

/* ---------------------------------------------------------------------------------------------
 * SharedMap last-writer-wins (MapKernel sequenced path, mapKernel.ts:706-853)
 * ------------------------------------------------------------------------------------------- */
/* Stage a batch into HBM (the one host→device crossing). Together with fmt_map_run this replaces
 * SharedMap.processMessagesCore (map/src/map.ts:288-311) → MapKernel.tryProcessMessage
 * (map/src/mapKernel.ts:619-630) for every sequenced set/delete/clear of every document, applied
 * in seq order (remote handlers mapKernel.ts:708-850). ops of document d are
 * ops[doc_op_offsets[d] .. doc_op_offsets[d+1]) in seq order; key ids < key_bound. Up to 2560
 * key ids the per-key tables live in LDS; larger key_bound takes the HBM-table kernel (2 * key_bound
 * u32 of device scratch per document, owned by the ctx). */
int fmt_map_load(fmt_ctx* ctx, const fmt_map_op* ops, uint64_t n_ops,
                 const uint64_t* doc_op_offsets, uint32_t n_docs, uint32_t key_bound);
/* Replay the staged batch (asynchronous on the ctx stream). */
int fmt_map_run(fmt_ctx* ctx);
/* Copy results to host: out[d * key_bound + k]. Synchronizes the ctx stream. Replaces reading
 * MapKernel.sequencedData (mapKernel.ts:131) for get()/summarizeCore (map.ts:176-246). */
int fmt_map_fetch(fmt_ctx* ctx, fmt_map_slot* out);
/* Zero-copy variant on caller-owned DEVICE buffers (e.g. torch tensors), launched on the ctx stream.
 * For key_bound > 2560 (the HBM-table path) d_out must be 8-byte aligned (FMT_E_USAGE otherwise).
 * Bad key ids (>= key_bound) are reported by fmt_map_check. */
int fmt_map_replay_device(fmt_ctx* ctx, const fmt_map_op* d_ops, const uint64_t* d_doc_op_offsets,
                          uint32_t n_docs, uint32_t key_bound, fmt_map_slot* d_out);
/* Synchronizes the ctx stream; FMT_E_DATA when an op of the last map run referenced a key id
 * >= key_bound (the remote op the reference would reject while processing it, mapKernel.ts:619-630). */
int fmt_map_check(fmt_ctx* ctx);

/* Sparse LWW for key pools of any size (key_bound up to 2^32 - 1): the per-key reductions run in
 * a per-document LDS hash table and the result is one entry per LIVE key, in JS Map insertion order
 * (birth seq ascending; map.ts:176-246 orders array-index keys first on top of that). Limits per
 * document: FMT_MAP_SPARSE_MAX_KEYS distinct keys and FMT_MAP_SPARSE_MAX_OPS ops (beyond them the
 * document gets no entries and fmt_map_fetch_sparse returns FMT_E_CAPACITY). */
typedef struct fmt_map_entry {
  uint32_t key;
  uint32_t value;      /* value id (FMT_MAP_VALUE_UNDEFINED: set with value undefined) */
  uint32_t birth_seq;  /* seq of the first set after the key's last delete/clear */
} fmt_map_entry;
#define FMT_MAP_SPARSE_MAX_KEYS 2048
#define FMT_MAP_SPARSE_MAX_OPS 16384
/* Stage a batch for the sparse path (no dense per-(doc, key) output is allocated). */
int fmt_map_load_sparse(fmt_ctx* ctx, const fmt_map_op* ops, uint64_t n_ops,
                        const uint64_t* doc_op_offsets, uint32_t n_docs, uint32_t key_bound);
/* Replay it (asynchronous on the ctx stream). */
int fmt_map_run_sparse(fmt_ctx* ctx);
/* counts[d] = live entries of document d (n_docs entries); entries of all documents packed in
 * document order into `entries` (cap_entries; *n_entries = their total). Synchronizes. */
int fmt_map_fetch_sparse(fmt_ctx* ctx, uint32_t* counts, fmt_map_entry* entries, uint64_t cap_entries,
                         uint64_t* n_entries);

/* Local-client pending state (the optimistic view of a client with unacknowledged local ops):
 * MapKernel.pendingData (mapKernel.ts:132-139) built by set / delete / clear (:388-538), emptied
 * by the local branches of the message handlers (:706-853) and by rollback (:633-700); read by
 * get / has (:374-392) and the iterator (:176-240). Each document's local-client events, in the
 * order they happened (the sequenced stream itself, local ops included, stays the document's
 * fmt_map_op records): */
#define FMT_MAP_EV_SUBMIT 0u   /* set / delete / clear of an attached map: the op enters pendingData */
#define FMT_MAP_EV_ACK 1u      /* the oldest unacknowledged submission came back sequenced
                                  (tryProcessMessage with local = true) and leaves pendingData */
#define FMT_MAP_EV_ROLLBACK 2u /* rollback of the newest unacknowledged submission */
typedef struct fmt_map_local_op {
  uint32_t doc;
  uint32_t key;        /* key id (set / delete); 0 for clear */
  uint32_t event;      /* FMT_MAP_EV_* */
  uint32_t kind_value; /* (kind << 30) | value id, as fmt_map_op. ACK / ROLLBACK repeat the op they
                          resolve, which must be the oldest / newest unacknowledged submission (the
                          reference asserts 0xbf2-0xbf9), else the document fails with FMT_E_DATA */
} fmt_map_local_op;
/* birth_seq of an optimistic entry that comes from a pending set lifetime: this bit | the index,
 * within the document's events, of the submission that created the lifetime */
#define FMT_MAP_PENDING_BIRTH 0x80000000u
/* Local events per document: one device thread walks a document's pending lists (a submit's
 * findLast and the iterator's scans are linear in the pending list), so a longer event list gets
 * status FMT_E_CAPACITY and no entries instead of stalling the launch. */
#define FMT_MAP_PENDING_MAX_EVENTS 16384
/* Every document's optimistic view over the sequenced entries of the last fmt_map_run_sparse and
 * the documents' local events (document d's at events[doc_event_offsets[d] .. [d + 1])), one
 * device thread per document. Asynchronous on the ctx stream. */
int fmt_map_pending_run(fmt_ctx* ctx, const fmt_map_local_op* events, uint64_t n_events,
                        const uint64_t* doc_event_offsets);
/* counts[d] = optimistic entries of document d; entries packed in document order, each document's
 * in internalIterator order (key, optimistic value, birth_seq: the sequenced birth, or
 * FMT_MAP_PENDING_BIRTH | creating submission); status[d] (may be NULL): FMT_OK, FMT_E_DATA for
 * a document whose ACK / ROLLBACK events do not match its pending ops, or FMT_E_CAPACITY for one
 * with more than FMT_MAP_PENDING_MAX_EVENTS events (no entries). Synchronizes. */
int fmt_map_pending_fetch(fmt_ctx* ctx, uint32_t* counts, int32_t* status, fmt_map_entry* entries,
                          uint64_t cap_entries, uint64_t* n_entries);

/* ---------------------------------------------------------------------------------------------
 * merge-tree / SharedString (Client.applyMsg observer path + zamboni, client.ts:1358-1391)
 * ------------------------------------------------------------------------------------------- */
/* Stage a batch into HBM. With fmt_mt_run this replaces SharedSegmentSequence.processMessagesCore
 * (sequence/src/sequence.ts:873-919) → Client.applyMsg (merge-tree/src/client.ts:1358-1379) for
 * every sequenced insert/remove/annotate/group message of every document (remote, observer view),
 * including updateSeqNumbers/setMinSeq (client.ts:1381-1391, mergeTree.ts:1147-1166) and zamboni
 * (zamboni.ts:33-213). Per-document errors land in fmt_mt_doc_result.status / fail_seq. */
int fmt_mt_load(fmt_ctx* ctx, const fmt_mt_batch* batch);
/* Replays every loaded document and returns when it is done. Plain batches start in the compact tier
 * (256 leaves, 2048 UTF-16 units); a document about to outgrow a tier stops at an op boundary, saves
 * its state, and the next tier resumes it: the small tier (512 leaves, 6144 units), then the large
 * tier (2048 leaves, 131071 units, text in HBM). Batches with obliterates or remove-order recording
 * start in the small tier, and a document that overflows inside an op replays again from its
 * inputs in the next tier. Stats cover every launch. */
int fmt_mt_run(fmt_ctx* ctx);
/* Per-document result headers for all docs (n_docs entries). Synchronizes the ctx stream. */
int fmt_mt_fetch_headers(fmt_ctx* ctx, fmt_mt_doc_result* out);
/* One document's leaves (cap_leaves), chars (cap_chars) and prop sets (cap_props): the converged
 * segment list that getText (MergeTreeTextHelper.ts:28-87) and Client.summarize
 * (client.ts:1548-1587, snapshotlegacy.ts:195-262) read. */
int fmt_mt_fetch_doc(fmt_ctx* ctx, uint32_t doc, fmt_mt_leaf* leaves, uint32_t cap_leaves,
                     uint16_t* chars, uint32_t cap_chars, fmt_mt_propset* props, uint32_t cap_props);
/* One document's catch-up ranges (header n_catchup entries, at most cap), in op order. Replaces the
 * messagesSinceMSNChange contents SharedSegmentSequence stashes for the legacy summary's catchupOps
 * blob (sequence.ts:949-1018, snapshotlegacy.ts:178-190). */
int fmt_mt_fetch_catchup(fmt_ctx* ctx, uint32_t doc, fmt_mt_catchup_range* out, uint32_t cap);
/* Every document's catch-up ranges in one device -> host copy, for the bulk summary path (what
 * summarizeMergeTree hands SnapshotLegacy for each string, sequence.ts:949-964, emitted as the
 * catchupOps blob, snapshotlegacy.ts:178-190): offsets[n_docs + 1] (packed prefix of the headers'
 * n_catchup) and, when out is not NULL, the ranges of document d at out[offsets[d] .. offsets[d+1]).
 * FMT_E_USAGE when cap < offsets[n_docs]. */
int fmt_mt_fetch_catchup_all(fmt_ctx* ctx, uint64_t* offsets, fmt_mt_catchup_range* out, uint64_t cap);
/* One document's remove-order entries (header n_rm_order entries, at most cap), in recording order:
 * with the first remover they give SnapshotV1's removedClientIds (snapshotV1.ts:235-250). */
int fmt_mt_fetch_remove_order(fmt_ctx* ctx, uint32_t doc, fmt_mt_remove_order* out, uint32_t cap);
/* One document's computed numbers (annotate-adjust results, FMT_MT_VALUE_COMPUTED + index): *n_out
 * = their count, the first min(count, cap) copied to out. */
int fmt_mt_fetch_numbers(fmt_ctx* ctx, uint32_t doc, double* out, uint32_t cap, uint32_t* n_out);
/* One document's per-leaf prop-set ids of getAtSeq(properties, minSeq) (segmentPropertiesManager.ts:328-344),
 * what the legacy summary reads (snapshotlegacy.ts:211-212); the first min(n_leaves, cap). Without
 * annotate-adjust in the batch they are the leaves' own props. */
int fmt_mt_fetch_legacy_props(fmt_ctx* ctx, uint32_t doc, uint16_t* out, uint32_t cap);
/* One document's remove clients with short ids 64..127 per leaf (bit c - 64), the first
 * min(n_leaves, cap) leaves: the rest of each leaf's remove-client set beyond fmt_mt_leaf.rm_clients
 * (getOrAddShortClientId interns without bound, client.ts:831-855). Zero for documents that no such
 * client touched. fmt_mt_state_digest folds them in (tag 10). */
int fmt_mt_fetch_rm_clients_hi(fmt_ctx* ctx, uint32_t doc, uint64_t* out, uint32_t cap);
/* The same for short ids 128..253 (round 6): two words per leaf, ids 128..191 (bit c - 128) then
 * 192..253 (bit c - 192), the first min(n_leaves, cap / 2) leaves. fmt_mt_state_digest folds them in
 * (tags 11, 12). */
int fmt_mt_fetch_rm_clients_hi2(fmt_ctx* ctx, uint32_t doc, uint64_t* out, uint32_t cap);
/* f4: one document's regenerated ops after the last fmt_mt_run, what regeneratePendingOp returned at
 * each FMT_MT_F_REGEN record in order (client.ts:1452-1542; replaces Client.regeneratePendingOp as the
 * host's resubmit source). Each op: type, pos1 / pos2 in the reconnect view, seq = the pending op's
 * localSeq, ref_seq = the document's currentSeq at the reconnect; an INSERT's payload / length (len +
 * FMT_MT_F_LEN_HI bits) address `text`, its pos2 and FMT_MT_F_MARKER flag are the original op's; an
 * ANNOTATE's payload is the original props op. *n_ops / *n_text = the counts, the first min(count,
 * cap) copied. Zero without local records. */
int fmt_mt_fetch_regen(fmt_ctx* ctx, uint32_t doc, fmt_mt_op* ops, uint32_t cap_ops, uint16_t* text, uint32_t cap_text,
                       uint32_t* n_ops, uint32_t* n_text);
/* Per-document 64-bit content digest of the converged state of the last fmt_mt_run (n_docs entries):
 * everything the reference's getText / summarize read back (MergeTreeTextHelper.ts:28-87,
 * snapshotlegacy.ts:195-262) — every leaf in document order with its stamps, remove-client set, length,
 * parent block ordinal and marker bit, its properties by value, the text — plus the header's collab
 * window, counts, depth and visible length; a failed document digests its status and fail_seq only.
 * Definition: mix(Σ elem(tag, index, word) mod 2^64), mix = the splitmix64 finalizer.
 * No reference counterpart: it lets a host check a whole batch against another replay (a replica, a
 * CPU client) without copying the state back. Synchronizes the ctx stream. */
int fmt_mt_state_digest(fmt_ctx* ctx, uint64_t* out);
/* Per-document capacities of this engine build (leaves, chars, prop sets): the large tier's, which
 * is where a document that outgrows the small tier ends up. */
int fmt_mt_capacity(uint32_t* max_leaves, uint32_t* max_chars, uint32_t* max_props);

#ifdef __cplusplus
}
#endif
#endif /* FMT_H_ */
