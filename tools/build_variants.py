#!/usr/bin/env python3
"""Build experimental variants of libfmt.so (source edits applied to a copy of csrc/) into
build/variants/<name>/libfmt.so, for same-process A/B timing with tools/bench_variants.py."""
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "fluidframework_amd", "csrc")


def _export_rev(rev, root):
    """csrc/ and include/fmt.h as of git revision `rev` (a committed engine version to A/B against)."""
    for rel in ("fluidframework_amd/csrc", "include"):
        files = subprocess.run(["git", "ls-tree", "-r", "--name-only", rev, rel], cwd=REPO, check=True,
                               capture_output=True, text=True).stdout.split()
        for f in files:
            if "/gen/" in f:
                continue
            dst = os.path.join(root, f)
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            data = subprocess.run(["git", "show", f"{rev}:{f}"], cwd=REPO, check=True, capture_output=True).stdout
            open(dst, "wb").write(data)


def build(name, edits, rev=None, flags=()):
    root = os.path.join(REPO, "build", "variants", name)
    csrc = os.path.join(root, "fluidframework_amd", "csrc")
    shutil.rmtree(root, ignore_errors=True)
    if rev:
        _export_rev(rev, root)
    else:
        shutil.copytree(SRC, csrc, ignore=shutil.ignore_patterns("gen"))
        os.makedirs(os.path.join(root, "include"), exist_ok=True)
        shutil.copy(os.path.join(REPO, "include", "fmt.h"), os.path.join(root, "include", "fmt.h"))
    for fname, old, new in edits:
        p = os.path.join(csrc, fname)
        s = open(p).read()
        assert old in s, (name, fname, old[:50])
        open(p, "w").write(s.replace(old, new))
    # kernels the variants do not touch link from the in-tree build (make -C fluidframework_amd/csrc);
    # VARIANT_ONLY=a.hip,b.hip compiles only those of the rest (the others from the in-tree build too)
    objs = [os.path.join(REPO, "build", "fmt", f) for f in ("map_lww.o", "map_sparse.o", "map_pending.o", "summary.o", "digest.o", "transfer.o")]
    only = [x for x in os.environ.get("VARIANT_ONLY", "").split(",") if x]
    procs = []
    for f in ["runtime.cpp", "mergetree.hip", "mergetree_compact.hip", "mergetree_large.hip", "mergetree_local.hip", "hugedoc.hip"]:
        if only and f not in only:
            objs.append(os.path.join(REPO, "build", "fmt", f.split(".")[0] + ".o"))
            continue
        o = os.path.join(root, f + ".o")
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-variable",
               *flags, "-x", "hip", "-c", "-o", o, os.path.join(csrc, f)]
        procs.append(subprocess.Popen(cmd))
        objs.append(o)
    for pr in procs:
        if pr.wait() != 0:
            raise SystemExit(f"{name}: compile failed")
    out = os.path.join(root, "libfmt.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o", out] + objs, check=True)
    if os.environ.get("NO_REPORT"):  # (skip the compact tier's resource report: minutes per variant)
        print(name, "| built")
        return out
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-Wno-unused-variable", *flags,
                        "-c", "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage",
                        os.path.join(csrc, "mergetree_compact.hip")], capture_output=True, text=True)
    info = [l.split("remark:")[1].strip() for l in r.stderr.splitlines()
            if "remark" in l and any(k in l for k in ("VGPRs:", "AGPRs", "Scratch", "Occupancy", "Spill"))]
    print(name, "|", "; ".join(info))
    return out


_LB = "return launchTier<false, S, false, kMtWaves, 2>(batch, out, docList, count, esc, numCUs, stream);"
LB1 = ("mergetree.hip", _LB, _LB.replace("kMtWaves, 2>", "kMtWaves, 1>"))
LB3 = ("mergetree.hip", _LB, _LB.replace("kMtWaves, 2>", "kMtWaves, 3>"))
LB4 = ("mergetree.hip", _LB, _LB.replace("kMtWaves, 2>", "kMtWaves, 4>"))
NODPP = ("wave.h", "#define FMT_USE_DPP 1", "#define FMT_USE_DPP 0")

NOFENCE = ("wave.h", """FMT_DEV void waveSync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}""", """FMT_DEV void waveSync() { asm volatile("" ::: "memory"); }""")

PROF = ("mt_engine.h", "#define FMT_PROFILE 0", "#define FMT_PROFILE 1")

# SharedMap kernel variants
MAP_NT = ("map_lww.hip", "if (u * 64u < n && i < n) rec[u] = recs[begin + i];",
          """if (u * 64u < n && i < n) {
          typedef unsigned int v4u __attribute__((ext_vector_type(4)));
          const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(recs + begin + i));
          rec[u] = make_uint4(v.x, v.y, v.z, v.w);
        }""")
MAP_W8 = ("map_lww.hip", "constexpr int kWaves = 4;", "constexpr int kWaves = 8;")
MAP_W2 = ("map_lww.hip", "constexpr int kWaves = 4;", "constexpr int kWaves = 2;")
MAP_LB2 = ("map_lww.hip", "__launch_bounds__(64 * kWaves) void mapLwwKernel", "__launch_bounds__(64 * kWaves, 2) void mapLwwKernel")

ROWS4 = [("mt_engine.h", "  static constexpr int kRows = 8;          // rows of 64 leaves (one VR element per row)",
          "  static constexpr int kRows = 4;          // rows of 64 leaves (one VR element per row)"),
         ("mt_engine.h", "  using VR = V8;\n};\n\nstruct LargeTier", "  using VR = V4;\n};\n\nstruct LargeTier")]

NOLOAD = ("mt_engine.h", "    if (in.loaded) loadSnapshot();", "    if (false) loadSnapshot();")

CW3 = ("mergetree_compact.hip", "launchTier<false, fmt_mt::CompactTier, false, kMtWavesCompact, 4>",
       "launchTier<false, fmt_mt::CompactTier, false, kMtWavesCompact, 3>")  # the round-2 occupancy

HW8 = [("huge_engine.h", "  static constexpr int kWaves = 4;", "  static constexpr int kWaves = 8;"),
       ("huge_engine.h", "  int32_t glN[4];", "  int32_t glN[8];")]

# the small tier's obliterate variant (escalated obliterate documents) at 1 wave/SIMD: 512 registers a
# wave, so its 32 spilled VGPRs go to AGPRs instead of scratch memory
OB_S1 = ("mergetree.hip", "    return launchTier<true, S, false, kMtWaves, 2>(batch, out, esc2 + 1, count, esc, numCUs, stream, esc2, n1);",
         "    return launchTier<true, S, false, kMtWaves, 1>(batch, out, esc2 + 1, count, esc, numCUs, stream, esc2, n1);")

# op records and insert text through a wave-uniform base (SGPRs) plus a small lane offset, so the
# loads take the saddr form and neither the loop index nor the arena pointers live in VGPRs (the
# compact kernel kept `in.ops` as a VGPR pair, spilled it, and its reload's vmcnt(0) waited for the
# next op's text prefetch every op)
FETCH_UNI = [("mt_engine.h", """    if (i < in.end) {
      const uint32_t* p = reinterpret_cast<const uint32_t*>(in.ops + i);
      FOR_LANES(l) { LANE(x) = l < 8 ? p[l] : 0u; }
    } else {""", """    if (i < in.end) {
      const uint32_t k = uni(static_cast<uint32_t>(i - in.begin));  // (documents below 2^32 ops)
      const uint32_t* p = reinterpret_cast<const uint32_t*>(in.ops + in.begin) + static_cast<uint64_t>(k) * 8u;
      FOR_LANES(l) { LANE(x) = l < 8 ? p[l] : 0u; }
    } else {"""),
             ("mt_engine.h", """    FOR_LANES(l) { LANE(x) = l < len ? static_cast<uint32_t>(in.text[payload + l]) : 0u; }
    return x;""", """    const uint16_t* t = in.text + uni(payload);
    FOR_LANES(l) { LANE(x) = l < len ? static_cast<uint32_t>(t[l]) : 0u; }
    return x;""")]

# the huge engine's rare paths (PropertiesManager records, remove order, relative positions, catch-up
# ranges) as out-of-line calls instead of force-inlined into the op loop
_COLD_FNS = ["void pmCompact(", "void pmUpdateMsn(", "void pmCopy(", "void pmDropLeaf(", "void pmAnnotate(",
             "void rmAppend(", "void rmFlush(", "int viewStart(", "int posFromRelativePos(", "bool resolveRelative(",
             "void recordCatchup(", "void pmLegacyProps("]
COLD = [("wave.h", "#define FMT_DEV __device__ __forceinline__",
         "#define FMT_DEV __device__ __forceinline__\n#define FMT_COLD __device__ __attribute__((noinline))"),
        ("wave.h", "#define FMT_DEV inline\n", "#define FMT_DEV inline\n#define FMT_COLD inline\n")] + \
       [("huge_engine.h", "  FMT_DEV " + f, "  FMT_COLD " + f) for f in _COLD_FNS]

# chars moves 256 units per iteration (4 loads per lane in flight, one wave sync per 256) instead of 64
SHIFT4 = [("mt_engine.h", """    const int count = nChars - from;
    for (int top = count - 1; top >= 0; top -= 64) {
      Lane<uint32_t> v;
      FOR_LANES(l) {
        const int t = top - l;
        LANE(v) = t >= 0 ? chRead(from + t) : 0u;
      }
      waveSync();
      FOR_LANES(l) {
        const int t = top - l;
        if (t >= 0) chWrite(from + t + by, LANE(v));
      }
      waveSync();
    }""", """    const int count = nChars - from;
    for (int top = count - 1; top >= 0; top -= 256) {
      Lane<uint32_t> v[4];
      FOR_LANES(l) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int t = top - l - 64 * u;
          LANE(v[u]) = t >= 0 ? chRead(from + t) : 0u;
        }
      }
      waveSync();
      FOR_LANES(l) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int t = top - l - 64 * u;
          if (t >= 0) chWrite(from + t + by, LANE(v[u]));
        }
      }
      waveSync();
    }"""),
          ("mt_engine.h", """    for (int base = from; base < nChars; base += 64) {
      Lane<uint32_t> v;
      FOR_LANES(l) {
        const int t = base + l;
        LANE(v) = t < nChars ? chRead(t) : 0u;
      }
      waveSync();
      FOR_LANES(l) {
        const int t = base + l;
        if (t < nChars) chWrite(t - by, LANE(v));
      }
      waveSync();
    }""", """    for (int base = from; base < nChars; base += 256) {
      Lane<uint32_t> v[4];
      FOR_LANES(l) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int t = base + l + 64 * u;
          LANE(v[u]) = t < nChars ? chRead(t) : 0u;
        }
      }
      waveSync();
      FOR_LANES(l) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int t = base + l + 64 * u;
          if (t < nChars) chWrite(t - by, LANE(v[u]));
        }
      }
      waveSync();
    }""")]

VISBF = [("mt_engine.h", '  FMT_DEV void visLengths(int refSeq, int client, Lane<VR>& vis, int nr) const {\n    FOR_ROWS(r, 0, nr) {\n      FOR_LANES(l) {\n        const uint32_t w0 = LANE(W[0])[r];\n        const int32_t ins = static_cast<int32_t>(LANE(W[1])[r]);\n        const int32_t rm = static_cast<int32_t>(LANE(W[2])[r]);\n        const int32_t ic = fClient(LANE(W[4])[r]);\n        const bool present = (ins <= refSeq || ic == client) && !(rm <= refSeq || removedBy(l, r, client));\n        LANE(vis)[r] = present ? fLen(w0) : 0u;\n      }\n    }\n  }', '  FMT_DEV void visLengths(int refSeq, int client, Lane<VR>& vis, int nr) const {\n    // branch-free: every term is a 0/1 word in a VGPR (shifts of differences, which cannot overflow:\n    // stamps are in [0, 2^31)), so no lane masks are combined in scalar registers\n    const bool hiW = C::kWords > 5 && client >= 32;\n    const uint32_t sh = client < 0 ? 0u : static_cast<uint32_t>(client & 31);\n    const uint32_t cm = client < 0 ? 0u : 1u;\n    const uint32_t cl8 = static_cast<uint32_t>(client) & 0xFFu;\n    FOR_ROWS(r, 0, nr) {\n      FOR_LANES(l) {\n        const uint32_t w0 = LANE(W[0])[r];\n        const uint32_t ins = LANE(W[1])[r];\n        const uint32_t rm = LANE(W[2])[r];\n        const uint32_t insLE = ((static_cast<uint32_t>(refSeq) - ins) >> 31) ^ 1u;\n        const uint32_t rmLE = ((static_cast<uint32_t>(refSeq) - rm) >> 31) ^ 1u;\n        const uint32_t icEq = (((LANE(W[4])[r] >> 24) ^ cl8) - 1u) >> 31;\n        const uint32_t rmb = ((hiW ? LANE(W[C::kWords > 5 ? 5 : 3])[r] : LANE(W[3])[r]) >> sh) & cm;\n        const uint32_t present = (insLE | icEq) & ((rmLE | rmb) ^ 1u);\n        LANE(vis)[r] = fLen(w0) * present;\n      }\n    }\n  }')]

VARIANTS = {
    # f4 local batches' compact tier at 2 waves/SIMD (256 VGPRs: no spills) instead of 3
    "locCL": [("mergetree_local.hip", "#define FMT_LOCAL_PATH 2", "#define FMT_LOCAL_PATH 0")],
    "locSL": [("mergetree_local.hip", "#define FMT_LOCAL_PATH 2", "#define FMT_LOCAL_PATH 1")],
    "locCSL": [],
    # the local small tier at 1 wave/SIMD (512 registers with AGPRs: no spills) instead of 2
    "locW1": [("mergetree_local.hip",
               "return launchTier<false, S, false, kMtWavesLocal, 2, false, true>(batch, out, docList, count, esc, numCUs, stream, nullptr, n1);",
               "return launchTier<false, S, false, kMtWavesLocal, 1, false, true>(batch, out, docList, count, esc, numCUs, stream, nullptr, n1);")],
    "t3lat": [],  # (working tree: huge tier with its block count / flags loaded beside the leaf fields)
    # huge tier without its per-phase shader-clock reads (ProfScope's s_memtime pairs)
    "t3noclk": [("huge_engine.h", "    return __builtin_amdgcn_s_memtime();", "    return 0;")],
    "visbf": VISBF,
    "chars4": SHIFT4,
    "pass8": [("huge_engine.h", "  static constexpr int kPassU = 16;", "  static constexpr int kPassU = 8;")],
    "pass4": [("huge_engine.h", "  static constexpr int kPassU = 8;", "  static constexpr int kPassU = 4;")],
    "pass2": [("huge_engine.h", "  static constexpr int kPassU = 4;", "  static constexpr int kPassU = 2;")],
    "shift4": [("huge_engine.h", "  static constexpr int kShiftU = 8;", "  static constexpr int kShiftU = 4;")],
    "shift8": [("huge_engine.h", "  static constexpr int kShiftU = 16;", "  static constexpr int kShiftU = 8;")],
    "hcur": [],
    "grad": [],  # (working tree: graduation masks from one batched pass, removals from the top)
    "pass1": [("huge_engine.h", "  static constexpr int kPassU = 2;", "  static constexpr int kPassU = 1;")],
    "shift2": [("huge_engine.h", "  static constexpr int kShiftU = 4;", "  static constexpr int kShiftU = 2;")],
    # obliterate small tier: its small -> large checkpoint saved by run() after the op loop (as plain
    # batches do), not inside it
    "obsb": [("mt_engine.h", "          if constexpr (Ob) {\n            if constexpr (kSavesCkpt) saveCkpt(i);\n            else saveBig(i);\n          } else {\n            ckptNext = i;\n          }",
              "          if constexpr (Ob && kSavesCkpt) {\n            saveCkpt(i);\n          } else {\n            ckptNext = i;\n          }"),
             ("mt_engine.h", "      else if constexpr (!Ob && kSavesBig) saveBig(ckptNext);", "      else if constexpr (kSavesBig) saveBig(ckptNext);")],
    # huge tier: 8 waves per workgroup (2 per SIMD) share the window / slot passes
    "w8": [("huge_engine.h", "  int32_t glN[4];", "  int32_t glN[8];"),
           ("huge_engine.h", "  static constexpr int kWaves = 4;", "  static constexpr int kWaves = 8;")],
    "w2s4": [],  # (working tree: window pass 2 x 64, slot pass 4 x 64 records per wave step)
    "ptext": [("huge_engine.h", "    return loadWg((off < S.textLen ? S.base : static_cast<const FMT_HBM uint16_t*>(S.text)) + off);",
               "    return (off < S.textLen ? S.base : static_cast<const FMT_HBM uint16_t*>(S.text))[off];")],
    "shift4b": [("huge_engine.h", "  static constexpr int kShiftU = 8;", "  static constexpr int kShiftU = 4;")],
    "pass2b": [("huge_engine.h", "  static constexpr int kPassU = 4;", "  static constexpr int kPassU = 2;")],
    # huge tier: HBM state read with plain (unordered) loads instead of workgroup-scope atomic ones
    "plainrd": [("huge_engine.h", "  FMT_DEV static uint32_t rd(const uint32_t* p) { return loadWg(p); }\n  FMT_DEV static int32_t rd(const int32_t* p) { return loadWg(p); }\n  FMT_DEV static uint32_t ldu(const uint32_t* p) { return uni(loadWg(p)); }\n  FMT_DEV static int32_t ldi(const int32_t* p) { return uni(loadWg(p)); }",
                 "  FMT_DEV static uint32_t rd(const uint32_t* p) { return *p; }\n  FMT_DEV static int32_t rd(const int32_t* p) { return *p; }\n  FMT_DEV static uint32_t ldu(const uint32_t* p) { return uni(*p); }\n  FMT_DEV static int32_t ldi(const int32_t* p) { return uni(*p); }")],
    "heap2": [],  # (working tree: hole-moving heap sifts, both children read together)
    # obliterate cascade: the small tier at 1 wave/SIMD (512 registers a wave: the overflow in AGPRs)
    "ob_o1": [("mergetree.hip", "  if (obliterate)\n    return launchTier<true, S, false, kMtWaves, 2>(batch, out, esc2 + 1,",
               "  if (obliterate)\n    return launchTier<true, S, false, kMtWaves, 1>(batch, out, esc2 + 1,")],
    "ob_base": [],
    "gq": [],  # (working tree: HugeState / HugeInputs buffers typed as global memory)
    "cur2": [],
    "cold": COLD,
    "fetch_uni": FETCH_UNI,
    "ob_s1": [OB_S1],
    "hw8": HW8,
    "prof": [PROF],
    "cw3": [CW3],
    "noload": [NOLOAD],
    "base": [],
    "rmt": [],
    "rmt_cold": COLD,
    "cur": [],
    "sops": [("mt_engine.h", "#define FMT_SCALAR_OPS 0", "#define FMT_SCALAR_OPS 1")],
    "cw2": [("mergetree_compact.hip", "constexpr int kMtWavesCompact = 4;", "constexpr int kMtWavesCompact = 2;")],
    "cw1": [("mergetree_compact.hip", "constexpr int kMtWavesCompact = 4;", "constexpr int kMtWavesCompact = 1;")],
    "sw2": [("mergetree.hip", "constexpr int kMtWaves = 4;  // small tier: 4 documents per workgroup, 2 waves/SIMD",
             "constexpr int kMtWaves = 2;  // small tier: 4 documents per workgroup, 2 waves/SIMD")],
    "nofence": [NOFENCE],
    "lb1": [LB1],
    "lb3": [LB3],
    "lb4": [LB4],
    "nodpp": [NODPP],
    "rows4": ROWS4,
    "rows4_lb3": ROWS4 + [LB3],
    "map_nt": [MAP_NT],
    "map_w8": [MAP_W8],
    "map_w2": [MAP_W2],
    "map_lb2": [MAP_LB2],
    "map_nt_w8": [MAP_NT, MAP_W8],
    "map_nt_w2": [MAP_NT, MAP_W2],
    "map_nt_w16": [MAP_NT, ("map_lww.hip", "constexpr int kWaves = 4;", "constexpr int kWaves = 16;")],
    "map_nt_w1": [MAP_NT, ("map_lww.hip", "constexpr int kWaves = 4;", "constexpr int kWaves = 1;")],
}
# compiler-flag variants (scheduler strategies) of the current sources
FLAGS = {
    "trk": ["-mllvm", "-amdgpu-use-amdgpu-trackers"],
    "ilp": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
    "mclause": ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"],
    "bias100": ["-mllvm", "-amdgpu-schedule-metric-bias=100"],
    "relaxocc": ["-mllvm", "-amdgpu-schedule-relaxed-occupancy"],
    "lines": ["-gline-tables-only"],  # (line tables only: the same code, for PC-sample attribution)
}
REVS = {"r5nb": "41cb064", "r5w2s4": "9cd02c8", "r5plain": "140dfb5", "r5heap": "2d9f706", "r5gq": "79be899", "r5ck": "bb3640d", "r5wc": "75f92c9", "v1": "352970f", "head": "6b38e0f", "prev": "HEAD", "pre_ob": "4bc1b08", "r4start": "14023f9", "r4relpos": "b4d93d3",
        "r4pend": "4831c1d", "r4rm": "07be56c", "r4v1": "efa25af"}  # committed engines to A/B against


if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    for n in names:
        if n in REVS:
            build(n, [], rev=REVS[n])
        elif n in FLAGS:
            build(n, [], flags=FLAGS[n])
        else:
            build(n, VARIANTS[n])
