#!/usr/bin/env python3
"""Build experimental variants of libfmt.so (source edits applied to a copy of csrc/) into
build/variants/<name>/libfmt.so, for same-process A/B timing with tools/bench_variants.py."""
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "fluidframework_amd", "csrc")


def build(name, edits):
    root = os.path.join(REPO, "build", "variants", name)
    csrc = os.path.join(root, "fluidframework_amd", "csrc")
    shutil.rmtree(root, ignore_errors=True)
    shutil.copytree(SRC, csrc, ignore=shutil.ignore_patterns("gen"))
    os.makedirs(os.path.join(root, "include"), exist_ok=True)
    shutil.copy(os.path.join(REPO, "include", "fmt.h"), os.path.join(root, "include", "fmt.h"))
    for fname, old, new in edits:
        p = os.path.join(csrc, fname)
        s = open(p).read()
        assert old in s, (name, fname, old[:50])
        open(p, "w").write(s.replace(old, new))
    objs = []
    for f in ["runtime.cpp", "map_lww.hip", "mergetree.hip"]:
        o = os.path.join(root, f + ".o")
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-variable",
               "-x", "hip", "-c", "-o", o, os.path.join(csrc, f)]
        subprocess.run(cmd, check=True)
        objs.append(o)
    out = os.path.join(root, "libfmt.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o", out] + objs, check=True)
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-Wno-unused-variable",
                        "-c", "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage",
                        os.path.join(csrc, "mergetree.hip")], capture_output=True, text=True)
    info = [l.split("remark:")[1].strip() for l in r.stderr.splitlines()
            if "remark" in l and any(k in l for k in ("VGPRs:", "AGPRs", "Scratch", "Occupancy"))]
    print(name, "|", "; ".join(info))
    return out


LB2 = ("mergetree.hip", "__launch_bounds__(64 * kMtWaves)", "__launch_bounds__(64 * kMtWaves, 2)")
LB3 = ("mergetree.hip", "__launch_bounds__(64 * kMtWaves)", "__launch_bounds__(64 * kMtWaves, 3)")
NODPP = ("wave.h", "#define FMT_USE_DPP 1", "#define FMT_USE_DPP 0")

NOFENCE = ("wave.h", """FMT_DEV void waveSync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}""", """FMT_DEV void waveSync() { asm volatile("" ::: "memory"); }""")

PROF = ("mt_engine.h", "#define FMT_PROFILE 0", "#define FMT_PROFILE 1")

VARIANTS = {
    "prof": [PROF],
    "nofence": [NOFENCE],
    "base": [],
    "lb2_nodpp": [LB2, NODPP],
    "lb3": [LB3],
    "nolaunder": [("wave.h", 'FMT_DEV void launder(V8& v) { asm volatile("" : "+v"(v)); }',
                   "FMT_DEV void launder(V8&) {}")],
    "lb2": [LB2],
}

if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    for n in names:
        build(n, VARIANTS[n])
