"""Result comparison shared by the emulation (CPU) and GPU parity tests.

A document's converged state is compared field by field against the oracle: every leaf in document
order (tombstones included) with its insert/remove stamps, remove-client set, text, properties and
parent leaf-block ordinal, plus the collab window and tree depth. Properties are compared by value
(document-local prop-set ids are an implementation detail).
"""
import ctypes
import os
import subprocess

import numpy as np

from fluidframework_amd.native import (CATCHUP_DTYPE, DOC_RESULT_DTYPE, LEAF_DTYPE, PROPSET_DTYPE, RM_ORDER_DTYPE,
                                       batch_struct)

HERE = os.path.dirname(os.path.abspath(__file__))
EMU_PATH = os.path.join(HERE, "_build", "libmt_emu.so")
_emu = None


def _build_atomic(cmd, out, src):
    """Compile to a private file, then rename over `out`: parallel test workers that find the library
    stale at once never load one another's half-written output."""
    tmp = f"{out}.{os.getpid()}.tmp"
    subprocess.run(cmd + ["-o", tmp, src], check=True)
    os.replace(tmp, out)


def emu_lib():
    global _emu
    if _emu is None:
        src = os.path.join(HERE, "emu", "mt_emu.cpp")
        deps = [src, os.path.join(HERE, "..", "include", "fmt.h")] + [os.path.join(HERE, "..", "fluidframework_amd", "csrc", f) for f in ("mt_engine.h", "wave.h", "huge_ckpt.h", "adjust.h")]
        if not os.path.exists(EMU_PATH) or os.path.getmtime(EMU_PATH) < max(os.path.getmtime(d) for d in deps):
            os.makedirs(os.path.dirname(EMU_PATH), exist_ok=True)
            _build_atomic(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wno-unknown-pragmas"], EMU_PATH, src)
        L = ctypes.CDLL(EMU_PATH)
        L.emu_mt_replay.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                                                              ctypes.c_void_p, ctypes.c_uint32]
        L.emu_mt_capacity.argtypes = [ctypes.c_int] + [ctypes.POINTER(ctypes.c_uint32)] * 3
        L.emu_mt_numbers.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
        L.emu_mt_legacy_props.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
        L.emu_mt_replay_local.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int]
        L.emu_mt_regen.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                   ctypes.POINTER(ctypes.c_uint32)]
        L.emu_mt_replay_large_ckpt.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_uint32, ctypes.c_void_p]
        L.emu_huge_ckpt_words.restype = ctypes.c_uint32
        L.emu_mt_replay_large_ckpt_rm.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_uint32, ctypes.c_void_p]
        L.emu_mt_adj_slab.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                      ctypes.POINTER(ctypes.c_uint32)]
        _emu = L
    return _emu


_huge = {}


def huge_emu_lib(tiny_groups=False):
    """The huge-document engine (csrc/huge_engine.h, T3) under host emulation, with its index
    invariants checked after every op (FMT_HUGE_CHECK). tiny_groups: 16 slots per group, 8 at load,
    so that group splits and cross-group walks happen on small documents."""
    if tiny_groups not in _huge:
        name = "libhuge_emu_tiny.so" if tiny_groups else "libhuge_emu.so"
        path = os.path.join(HERE, "_build", name)
        src = os.path.join(HERE, "emu", "huge_emu.cpp")
        deps = [src, os.path.join(HERE, "..", "include", "fmt.h")] + [os.path.join(HERE, "..", "fluidframework_amd", "csrc", f) for f in ("huge_engine.h", "wave.h", "adjust.h", "huge_ckpt.h")]
        if not os.path.exists(path) or os.path.getmtime(path) < max(os.path.getmtime(d) for d in deps):
            os.makedirs(os.path.dirname(path), exist_ok=True)
            extra = ["-DFMT_HUGE_SLOTCAP=16", "-DFMT_HUGE_FILL=8"] if tiny_groups else []
            _build_atomic(["g++", "-O2", "-g", "-std=c++17", "-fPIC", "-shared", "-Wno-unknown-pragmas",
                           "-DFMT_HUGE_CHECK_BUILD"] + extra, path, src)
        L = ctypes.CDLL(path)
        L.emu_huge_replay.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                      ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        L.emu_huge_replay_rec.argtypes = L.emu_huge_replay.argtypes + [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                                                      ctypes.c_uint32]
        L.emu_huge_replay_adj.argtypes = L.emu_huge_replay_rec.argtypes + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                                          ctypes.c_void_p]
        L.emu_huge_replay_hi.argtypes = L.emu_huge_replay.argtypes + [ctypes.c_void_p]
        L.emu_huge_resume.argtypes = ([ctypes.c_void_p, ctypes.c_uint32] + [ctypes.c_void_p] * 6 +
                                      [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)])
        L.emu_huge_resume_adj.argtypes = ([ctypes.c_void_p, ctypes.c_uint32] + [ctypes.c_void_p] * 5 +
                                          [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                           ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64)])
        L.emu_huge_resume_rm.argtypes = ([ctypes.c_void_p, ctypes.c_uint32] + [ctypes.c_void_p] * 6 +
                                         [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)])
        _huge[tiny_groups] = L
    return _huge[tiny_groups]


def emu_huge_replay_adjust(batch, doc=0, tiny_groups=False, cap_props=65534):
    """(header, leaves, chars, props, legacy prop sets per leaf, computed numbers) of document `doc`
    of an annotate-adjust batch replayed by the emulated huge engine."""
    from fluidframework_amd.native import DOC_RESULT_DTYPE, LEAF_DTYPE, PROPSET_DTYPE, batch_struct

    sd = batch.snapshots[doc] if batch.snapshots is not None else None
    segs = int(sd["n_header"]) + int(sd["n_body"]) if sd is not None and sd["loaded"] else 1
    nops = int(batch.doc_op_offsets[doc + 1] - batch.doc_op_offsets[doc])
    cap_leaves, cap_chars = segs + 3 * nops + 8, len(batch.text) + 8
    hdr = np.zeros(1, dtype=DOC_RESULT_DTYPE)
    leaves = np.zeros(cap_leaves, dtype=LEAF_DTYPE)
    chars = np.zeros(cap_chars, dtype="<u2")
    props = np.zeros(cap_props, dtype=PROPSET_DTYPE)
    legacy = np.zeros(cap_leaves, dtype="<u2")
    nums = np.zeros(1 << 16, dtype=np.float64)
    nn = ctypes.c_uint32()
    b, keep = batch_struct(batch)
    huge_emu_lib(tiny_groups).emu_huge_replay_adj(ctypes.addressof(b), doc, _p(hdr), _p(leaves), cap_leaves, _p(chars),
                                                  cap_chars, _p(props), None, 0, None, 0, _p(legacy), _p(nums),
                                                  len(nums), ctypes.byref(nn))
    del keep
    h = hdr[0]
    n = int(h["n_leaves"])
    return h, leaves[:n], chars[: int(h["n_chars"])], props[: int(h["n_props"])], legacy[:n], nums[: nn.value]


def emu_huge_replay(batch, doc=0, cap_leaves=None, cap_chars=None, tiny_groups=False, cap_catchup=0, cap_rm=0,
                    cap_props=65534):
    """(header, leaves, chars, props) of document `doc` replayed by the emulated huge engine, plus its
    catch-up ranges (header n_catchup of them) when cap_catchup > 0, then its remove-order entries
    (header n_rm_order of them) when cap_rm > 0."""
    from fluidframework_amd.native import (CATCHUP_DTYPE, DOC_RESULT_DTYPE, LEAF_DTYPE, PROPSET_DTYPE, RM_ORDER_DTYPE,
                                           batch_struct)

    sd = batch.snapshots[doc] if batch.snapshots is not None else None
    segs = int(sd["n_header"]) + int(sd["n_body"]) if sd is not None and sd["loaded"] else 1
    nops = int(batch.doc_op_offsets[doc + 1] - batch.doc_op_offsets[doc])
    cap_leaves = cap_leaves or segs + 3 * nops + 8
    cap_chars = cap_chars or len(batch.text) + 8
    hdr = np.zeros(1, dtype=DOC_RESULT_DTYPE)
    leaves = np.zeros(cap_leaves, dtype=LEAF_DTYPE)
    chars = np.zeros(cap_chars, dtype="<u2")
    props = np.zeros(cap_props, dtype=PROPSET_DTYPE)
    b, keep = batch_struct(batch)
    cu = np.zeros(max(cap_catchup, 1), dtype=CATCHUP_DTYPE)
    rm = np.zeros(max(cap_rm, 1), dtype=RM_ORDER_DTYPE)
    huge_emu_lib(tiny_groups).emu_huge_replay_rec(ctypes.addressof(b), doc, _p(hdr), _p(leaves), cap_leaves, _p(chars),
                                                  cap_chars, _p(props), _p(cu) if cap_catchup else None, cap_catchup,
                                                  _p(rm) if cap_rm else None, cap_rm)
    del keep
    h = hdr[0]
    out = h, leaves[: int(h["n_leaves"])], chars[: int(h["n_chars"])], props[: int(h["n_props"])]
    if cap_catchup:
        out = out + (cu[: int(h["n_catchup"])],)
    if cap_rm:
        out = out + (rm[: int(h["n_rm_order"])],)
    return out


def emu_huge_replay_hi(batch, doc=0, tiny_groups=False, cap_props=65534, hi2=False):
    """(header, leaves, chars, props, remove clients 64..127 per leaf[, (n, 2) remove clients 128..191
    and 192..253 with hi2]) of document `doc` replayed by the emulated huge engine with its side table
    for short ids 64..253."""
    from fluidframework_amd.native import DOC_RESULT_DTYPE, LEAF_DTYPE, PROPSET_DTYPE, batch_struct

    sd = batch.snapshots[doc] if batch.snapshots is not None else None
    segs = int(sd["n_header"]) + int(sd["n_body"]) if sd is not None and sd["loaded"] else 1
    nops = int(batch.doc_op_offsets[doc + 1] - batch.doc_op_offsets[doc])
    cap_leaves, cap_chars = segs + 3 * nops + 8, len(batch.text) + 8
    hdr = np.zeros(1, dtype=DOC_RESULT_DTYPE)
    leaves = np.zeros(cap_leaves, dtype=LEAF_DTYPE)
    chars = np.zeros(cap_chars, dtype="<u2")
    props = np.zeros(cap_props, dtype=PROPSET_DTYPE)
    hi = np.zeros((cap_leaves, 3), dtype=np.uint64)  # (huge_engine.h kHiOutWords per leaf)
    b, keep = batch_struct(batch)
    huge_emu_lib(tiny_groups).emu_huge_replay_hi(ctypes.addressof(b), doc, _p(hdr), _p(leaves), cap_leaves, _p(chars),
                                                 cap_chars, _p(props), _p(hi))
    del keep
    h = hdr[0]
    n = int(h["n_leaves"])
    out = h, leaves[:n], chars[: int(h["n_chars"])], props[: int(h["n_props"])], hi[:n, 0].copy()
    return out + (hi[:n, 1:].copy(),) if hi2 else out


def emu_grow_replay(batch, tiny_groups=False, cap_catchup=0, cap_rm=0):
    """The runtime's large → huge path under host emulation: the large tier over every document from
    its first op, each document it is about to outgrow stopping at its checkpoint (huge_ckpt.h), then
    the huge tier resuming it from there. Returns per document (header, leaves, chars, props[, catch-up
    ranges][, remove-order entries: cap_rm > 0][, legacy prop sets per leaf, computed numbers:
    annotate-adjust batches]) and the op index each resumed at (0: the large tier finished it)."""
    adjust = batch.adjusts is not None
    cl, cc, cp = emu_caps(True)
    n = batch.n_docs
    hdr = np.zeros(n, dtype=DOC_RESULT_DTYPE)
    leaves = np.zeros(n * cl, dtype=LEAF_DTYPE)
    chars = np.zeros(n * cc, dtype="<u2")
    props = np.zeros(n * cp, dtype=PROPSET_DTYPE)
    cu = np.zeros(max(n * cap_catchup, 1), dtype=CATCHUP_DTYPE)
    L = emu_lib()
    ck = np.zeros(n * int(L.emu_huge_ckpt_words()), dtype=np.uint32)
    b, keep = batch_struct(batch)
    rm = np.zeros(max(n * cap_rm, 1), dtype=RM_ORDER_DTYPE)
    if cap_rm:
        assert not cap_catchup and not adjust
        L.emu_mt_replay_large_ckpt_rm(ctypes.addressof(b), _p(hdr), _p(leaves), _p(chars), _p(props), _p(rm), cap_rm,
                                      _p(ck))
    else:
        L.emu_mt_replay_large_ckpt(ctypes.addressof(b), _p(hdr), _p(leaves), _p(chars), _p(props),
                                   _p(cu) if cap_catchup else None, cap_catchup, _p(ck))
    words = int(L.emu_huge_ckpt_words())
    out, resumed = [], []
    for d in range(n):
        if int(hdr[d]["status"]) != -35:  # (fmt_ckpt::kStatusHuge)
            h = hdr[d]
            res = (h, leaves[d * cl: d * cl + int(h["n_leaves"])], chars[d * cc: d * cc + int(h["n_chars"])],
                   props[d * cp: d * cp + int(h["n_props"])])
            if cap_catchup:
                res = res + (cu[d * cap_catchup: d * cap_catchup + int(h["n_catchup"])],)
            if cap_rm:
                res = res + (rm[d * cap_rm: d * cap_rm + int(h["n_rm_order"])],)
            if adjust:
                lg = emu_legacy_props(d)
                res = res + (lg[: int(h["n_leaves"])] if lg is not None else None, emu_numbers(d))
            out.append(res)
            resumed.append(0)
            continue
        sd = batch.snapshots[d] if batch.snapshots is not None else None
        segs = int(sd["n_header"]) + int(sd["n_body"]) if sd is not None and sd["loaded"] else 1
        nops = int(batch.doc_op_offsets[d + 1] - batch.doc_op_offsets[d])
        hcl, hcc = segs + 3 * nops + 8, len(batch.text) + 8 + int(batch.doc_init[d][1]) + cc
        h1 = np.zeros(1, dtype=DOC_RESULT_DTYPE)
        lv = np.zeros(hcl, dtype=LEAF_DTYPE)
        ch = np.zeros(hcc, dtype="<u2")
        pr = np.zeros(65534, dtype=PROPSET_DTYPE)
        cud = np.zeros(max(cap_catchup, 1), dtype=CATCHUP_DTYPE)
        if cap_catchup:
            cud[:cap_catchup] = cu[d * cap_catchup: (d + 1) * cap_catchup]
        at = ctypes.c_uint64(0)
        if adjust:
            assert not cap_catchup
            pm_recs = int(ck[d * words + 15])  # (fmt_ckpt::kPmN)
            pm = np.zeros(4 * max(pm_recs, 1), dtype=np.uint32)
            nums_in = np.zeros(4096, dtype=np.float64)
            n_in = ctypes.c_uint32(0)
            assert L.emu_mt_adj_slab(d, _p(pm), pm_recs, _p(nums_in), len(nums_in), ctypes.byref(n_in)) == 0
            legacy = np.zeros(hcl, dtype="<u2")
            nums = np.zeros(1 << 16, dtype=np.float64)
            nn = ctypes.c_uint32(0)
            huge_emu_lib(tiny_groups).emu_huge_resume_adj(
                ctypes.addressof(b), d, _p(ck[d * words:]), _p(leaves[d * cl:]), _p(chars[d * cc:]), _p(props[d * cp:]),
                _p(pm), pm_recs, _p(nums_in), n_in.value, _p(h1), _p(lv), hcl, _p(ch), hcc, _p(pr), _p(legacy),
                _p(nums), len(nums), ctypes.byref(nn), ctypes.byref(at))
        elif cap_rm:
            rmd = rm[d * cap_rm: (d + 1) * cap_rm].copy()
            huge_emu_lib(tiny_groups).emu_huge_resume_rm(
                ctypes.addressof(b), d, _p(ck[d * words:]), _p(leaves[d * cl:]), _p(chars[d * cc:]), _p(props[d * cp:]),
                _p(h1), _p(lv), hcl, _p(ch), hcc, _p(pr), _p(rmd), cap_rm, ctypes.byref(at))
        else:
            huge_emu_lib(tiny_groups).emu_huge_resume(
                ctypes.addressof(b), d, _p(ck[d * words:]), _p(leaves[d * cl:]), _p(chars[d * cc:]), _p(props[d * cp:]),
                _p(h1), _p(lv), hcl, _p(ch), hcc, _p(pr), _p(cud) if cap_catchup else None, cap_catchup, ctypes.byref(at))
        h = h1[0]
        res = (h, lv[: int(h["n_leaves"])], ch[: int(h["n_chars"])], pr[: int(h["n_props"])])
        if cap_catchup:
            res = res + (cud[: int(h["n_catchup"])],)
        if cap_rm:
            res = res + (rmd[: int(h["n_rm_order"])],)
        if adjust:
            res = res + (legacy[: int(h["n_leaves"])], nums[: nn.value])
        out.append(res)
        resumed.append(int(at.value))
    del keep
    return out, resumed


def oracle_rm_clients_hi2(batch, doc, n_leaves):
    """The oracle's remove clients 128..191 and 192..253 per final leaf ((n, 2), from every remove stamp)."""
    import oracle

    hi = np.zeros((n_leaves, 2), dtype=np.uint64)
    for leaf, stamps in oracle.mt_removers(batch, doc).items():
        for client, _, _ in stamps:
            if 128 <= client < 256:
                hi[leaf, (client - 128) // 64] |= np.uint64(1) << np.uint64((client - 128) % 64)
    return hi


def oracle_rm_clients_hi(batch, doc, n_leaves):
    """The oracle's remove clients 64..127 per final leaf (from every remove stamp, oracle.mt_removers)."""
    import oracle

    hi = np.zeros(n_leaves, dtype=np.uint64)
    for leaf, stamps in oracle.mt_removers(batch, doc).items():
        for client, _, _ in stamps:
            if 64 <= client < 128:
                hi[leaf] |= np.uint64(1) << np.uint64(client - 64)
    return hi


def emu_caps(large=False):
    a, b, c = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    emu_lib().emu_mt_capacity(int(large), ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
    return a.value, b.value, c.value


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def emu_replay(batch, cap_catchup=0, force_ob=False, large=False, cap_rm=0):
    """Run the engine source under host emulation (small tier, or the large tier the runtime replays
    overflowing documents in); returns (headers, leaves, chars, props), plus the catch-up ranges
    (n_docs, cap_catchup) when cap_catchup > 0, then the remove-order entries (n_docs, cap_rm) when
    cap_rm > 0."""
    cl, cc, cp = emu_caps(large)
    n = batch.n_docs
    hdr = np.zeros(n, dtype=DOC_RESULT_DTYPE)
    leaves = np.zeros(n * cl, dtype=LEAF_DTYPE)
    chars = np.zeros(n * cc, dtype="<u2")
    props = np.zeros(n * cp, dtype=PROPSET_DTYPE)
    cu = np.zeros(n * cap_catchup, dtype=CATCHUP_DTYPE) if cap_catchup else None
    rm = np.zeros(n * cap_rm, dtype=RM_ORDER_DTYPE) if cap_rm else None
    b, keep = batch_struct(batch)
    emu_lib().emu_mt_replay(ctypes.addressof(b), _p(hdr), _p(leaves), _p(chars), _p(props),
                            _p(cu) if cu is not None else None, cap_catchup, int(force_ob), int(large),
                            _p(rm) if rm is not None else None, cap_rm)
    del keep
    out = (hdr, leaves.reshape(n, cl), chars.reshape(n, cc), props.reshape(n, cp))
    if cap_catchup:
        out = out + (cu.reshape(n, cap_catchup),)
    if cap_rm:
        out = out + (rm.reshape(n, cap_rm),)
    return out


def emu_replay_local(batch, large_only=False, compact_first=False):
    """f4 batches (local submissions / acks / rollbacks / reconnects) under host emulation, as the
    runtime runs them: the small tier's local variant, then the large tier's for the documents it
    could not hold (large_only: every document in the large tier; compact_first: the compact tier's
    local variant first, then the small and the large tier's). (headers, leaves, chars, props) at
    large-tier strides."""
    cl, cc, cp = emu_caps(True)
    n = batch.n_docs
    hdr = np.zeros(n, dtype=DOC_RESULT_DTYPE)
    leaves = np.zeros(n * cl, dtype=LEAF_DTYPE)
    chars = np.zeros(n * cc, dtype="<u2")
    props = np.zeros(n * cp, dtype=PROPSET_DTYPE)
    b, keep = batch_struct(batch)
    emu_lib().emu_mt_replay_local(ctypes.addressof(b), _p(hdr), _p(leaves), _p(chars), _p(props), 1 if large_only else 3 if compact_first else 0)
    del keep
    return hdr, leaves.reshape(n, cl), chars.reshape(n, cc), props.reshape(n, cp)


def emu_regen(doc: int):
    """Document `doc`'s regenerated ops and their text after the last emu_replay_local."""
    from fluidframework_amd.streams import MT_OP_DTYPE

    ops = np.zeros(4096, dtype=MT_OP_DTYPE)
    text = np.zeros(1 << 16, dtype="<u2")
    nt = ctypes.c_uint32(0)
    n = emu_lib().emu_mt_regen(doc, _p(ops), len(ops), _p(text), len(text), ctypes.byref(nt))
    return ops[: max(n, 0)], text[: nt.value]


def emu_legacy_props(doc: int):
    """Document `doc`'s per-leaf getAtSeq(minSeq) prop sets after the last emu_replay of a batch with
    annotate-adjust (None otherwise)."""
    out = np.zeros(4096, dtype=np.uint16)
    n = emu_lib().emu_mt_legacy_props(doc, _p(out), 4096)
    return out[:n] if n else None


def emu_numbers(doc: int) -> np.ndarray:
    """Document `doc`'s computed annotate-adjust numbers after the last emu_replay."""
    out = np.zeros(4096, dtype=np.float64)
    n = emu_lib().emu_mt_numbers(doc, _p(out), 4096)
    return out[:n]


def resolve_props(pid, table):
    from fluidframework_amd.native import propset_entries

    if pid == 0xFFFF:
        return None
    return propset_entries(table, pid)


HEADER_FIELDS = ["status", "cur_seq", "min_seq", "n_leaves", "n_chars", "n_blocks", "depth", "visible_len"]
LEAF_FIELDS = ["ins_seq", "rm_seq", "rm_clients", "char_off", "len", "ins_client", "block", "pad"]


def compare_doc(exp, got):
    """exp/got = (header, leaves[:n], chars[:n_chars], props[:n_props]); returns a list of diffs."""
    eh, el, ec, ep = exp
    gh, gl, gc, gp = got
    diffs = []
    for f in HEADER_FIELDS:
        if int(eh[f]) != int(gh[f]):
            diffs.append(f"header.{f}: expected {int(eh[f])} got {int(gh[f])}")
    if diffs:
        return diffs
    n = int(eh["n_leaves"])
    for f in LEAF_FIELDS:
        bad = np.nonzero(el[f][:n] != gl[f][:n])[0]
        if len(bad):
            i = int(bad[0])
            diffs.append(f"leaf[{i}].{f}: expected {el[f][i]} got {gl[f][i]}")
    ep_res = [resolve_props(int(p), ep) for p in el["props"][:n]]
    gp_res = [resolve_props(int(p), gp) for p in gl["props"][:n]]
    for i, (a, b) in enumerate(zip(ep_res, gp_res)):
        if a != b:
            diffs.append(f"leaf[{i}].props: expected {a} got {b}")
            break
    nc = int(eh["n_chars"])
    if not np.array_equal(ec[:nc], gc[:nc]):
        i = int(np.nonzero(ec[:nc] != gc[:nc])[0][0])
        diffs.append(f"chars differ first at {i}")
    return diffs


def visible_text(hdr, leaves, chars):
    n = int(hdr["n_leaves"])
    out = []
    for L in leaves[:n]:
        if int(L["rm_seq"]) == 0x7FFFFFFF and not int(L["pad"]) & 0x8000:  # (markers: no text)
            o = int(L["char_off"])
            out.append(chars[o : o + int(L["len"])].tobytes().decode("utf-16-le", "surrogatepass"))
    return "".join(out)
