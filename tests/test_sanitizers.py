"""Host sanitizers over the oracle and the engine source (SURVEY.md §5's sanitizer counterpart).

tests/san/san_check.cpp links the oracle (oracle/*.cpp), the merge-tree engine under host emulation
(tests/emu/mt_emu.cpp: the same mt_engine.h the gfx950 kernels compile) and the conflict-farm
generator, built with -fsanitize=address,undefined (-fno-sanitize-recover: the first report aborts).
It replays generated documents through every engine tier and the compact → small → large
checkpoint cascade, and checks each document against the oracle. GPU-side sanitizers are not
available on this pool; this covers the host builds of the same sources.
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
BIN = os.path.join(HERE, "_build", "san_check")
SRCS = [os.path.join(HERE, "san", "san_check.cpp"), os.path.join(HERE, "emu", "mt_emu.cpp")] + \
       [os.path.join(REPO, "oracle", f) for f in ("mergetree.cpp", "map.cpp", "capi.cpp")] + \
       [os.path.join(REPO, "fluidframework_amd", "csrc", "gen", "fmtgen.cpp")]
DEPS = SRCS + [os.path.join(REPO, "include", "fmt.h")] + \
       [os.path.join(REPO, "fluidframework_amd", "csrc", f) for f in ("mt_engine.h", "wave.h")] + \
       [os.path.join(REPO, "oracle", f) for f in ("mergetree.hpp", "common.hpp", "map.hpp")]


def _build():
    if os.path.exists(BIN) and os.path.getmtime(BIN) >= max(os.path.getmtime(d) for d in DEPS):
        return
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-Wno-unknown-pragmas", "-o", BIN] + SRCS + ["-lpthread"], check=True)


def test_oracle_and_engine_source_under_asan_ubsan():
    _build()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [l for l in r.stdout.splitlines() if l.startswith("tier")]
    assert len(lines) == 7 and all(l.endswith(": 0 mismatches") for l in lines), r.stdout
