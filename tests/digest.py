"""The state digest restated in numpy: the definition both fmt_mt_state_digest (device,
csrc/digest.hip) and the oracle (oracle/capi.cpp digestOf) implement. Test-only."""
import numpy as np

from fluidframework_amd.native import propset_entries

M64 = (1 << 64) - 1


def _mix(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _elems(tag, idx, w):
    idx = np.asarray(idx, dtype=np.uint64)
    w = np.asarray(w, dtype=np.uint64)
    return _mix(_mix((np.uint64(tag) << np.uint64(56)) ^ idx) ^ w)


def _sum(a):
    return int(np.asarray(a, dtype=np.uint64).sum(dtype=np.uint64)) if np.size(a) else 0


def state_digest(hdr, leaves, chars, props, rm_hi=None, rm_hi2=None) -> int:
    """Digest of one document from its header, leaves[:n_leaves], chars[:n_chars] and prop sets."""
    u32 = lambda v: int(v) & 0xFFFFFFFF  # noqa: E731
    if int(hdr["status"]) != 0:
        acc = (_sum(_elems(1, [0], [u32(hdr["status"])])) + _sum(_elems(1, [1], [u32(hdr["fail_seq"])]))) & M64
        return int(_mix(np.uint64(acc)))
    f = [u32(hdr[k]) for k in ("status", "cur_seq", "min_seq", "n_leaves", "n_chars", "n_blocks", "depth", "visible_len")]
    acc = _sum(_elems(1, np.arange(8), f))
    n = int(hdr["n_leaves"])
    L = leaves[:n]
    i = np.arange(n, dtype=np.uint64)
    w2 = L["ins_seq"].astype(np.int64).astype(np.uint64) & np.uint64(0xFFFFFFFF)
    w2 |= (L["rm_seq"].astype(np.int64).astype(np.uint64) & np.uint64(0xFFFFFFFF)) << np.uint64(32)
    acc += _sum(_elems(2, i, w2))
    acc += _sum(_elems(3, i, L["rm_clients"]))
    acc += _sum(_elems(4, i, L["char_off"].astype(np.uint64) | (L["len"].astype(np.uint64) << np.uint64(32))))
    w5 = (L["ins_client"].astype(np.int64).astype(np.uint64) & np.uint64(0xFFFF)) | (L["block"].astype(np.uint64) << np.uint64(16))
    w5 |= L["pad"].astype(np.uint64) << np.uint64(32)
    acc += _sum(_elems(5, i, w5))
    for k in range(n):
        p = int(L["props"][k])
        if p == 0xFFFF:
            acc += _sum(_elems(6, [k], [M64]))
        else:
            m = int(props[p]["n"])
            acc += _sum(_elems(6, [k], [m]))
            kv = np.array(propset_entries(props, p), dtype=np.uint64)
            if m:  # entries 8.. of a wide set (several records) under tag 9
                acc += _sum(_elems(7, np.arange(min(m, 8)) + 8 * k, kv[:8]))
            if m > 8:
                acc += _sum(_elems(9, np.arange(8, m) + 64 * k, kv[8:]))
    if rm_hi is not None:  # remove clients 64..127 (tag 10), on the leaves that have any
        hi = np.asarray(rm_hi[:n], dtype=np.uint64)
        at = np.nonzero(hi)[0]
        if len(at):
            acc += _sum(_elems(10, at.astype(np.uint64), hi[at]))
    if rm_hi2 is not None:  # remove clients 128..191 (tag 11) and 192..253 (tag 12), (n, 2)
        hi2 = np.asarray(rm_hi2[:n], dtype=np.uint64).reshape(-1, 2)
        for k in range(2):
            at = np.nonzero(hi2[:, k])[0]
            if len(at):
                acc += _sum(_elems(11 + k, at.astype(np.uint64), hi2[at, k]))
    nc = int(hdr["n_chars"])
    acc += _sum(_elems(8, np.arange(nc), chars[:nc]))
    return int(_mix(np.uint64(acc & M64)))
