"""The N-API addon's lifetime and exit paths on the CPU.

fmt_napi.node is built here against a device-less stand-in for libfmt.so (tests/napi_exit/fmt_stub.cpp:
every fmt.h entry point, replays that replay nothing), both with AddressSanitizer, and node runs
tests/napi_exit/exit_driver.js under LD_PRELOAD=libasan with freed memory filled (a read through a
freed object then faults instead of silently reading stale bytes). Each run opens and closes contexts,
leaves some open for the env cleanup hook, keeps a replay pending at exit, creates thousands of dead
handles before a natural GC right before teardown, and runs worker_threads that open their own
contexts (a worker's teardown must close only its own; a handle used from another thread is refused).
200 runs must all exit 0 with no sanitizer report.
"""
import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "napi_exit")
OUT = os.path.join(REPO, "tests", "_build", "napi_exit")
NODE_API = "/usr/include/node/node_api.h"

pytestmark = pytest.mark.skipif(shutil.which("node") is None or not os.path.exists(NODE_API),
                                reason="node or node_api.h missing")


def _libasan():
    return subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True, check=True).stdout.strip()


@pytest.fixture(scope="module")
def addon():
    os.makedirs(OUT, exist_ok=True)
    common = ["g++", "-O1", "-g", "-std=c++17", "-shared", "-fPIC", "-fsanitize=address", "-fno-omit-frame-pointer",
              "-I" + os.path.join(REPO, "include")]
    subprocess.run(common + ["-o", os.path.join(OUT, "libfmt.so"), os.path.join(SRC, "fmt_stub.cpp")], check=True)
    subprocess.run(common + ["-Wall", "-DNODE_GYP_MODULE_NAME=fmt_napi", "-DNAPI_VERSION=8", "-I/usr/include/node",
                             "-o", os.path.join(OUT, "fmt_napi.node"),
                             os.path.join(REPO, "fluidframework_amd", "napi", "fmt_napi.cc"),
                             "-L" + OUT, "-lfmt", "-Wl,-rpath,$ORIGIN"], check=True)
    return os.path.join(OUT, "fmt_napi.node")


def _run(addon_path, asan=True, extra=None):
    env = dict(os.environ, FMT_NAPI_ADDON=addon_path)
    if asan:
        env["LD_PRELOAD"] = _libasan()
        env["ASAN_OPTIONS"] = "detect_leaks=0:max_free_fill_size=65536:free_fill_byte=190:abort_on_error=0"
    env.update(extra or {})
    p = subprocess.run(["node", "--expose-gc", os.path.join(SRC, "exit_driver.js")], env=env,
                       capture_output=True, text=True, timeout=120)
    return p.returncode, p.stdout, p.stderr


def test_stub_exports_every_declared_entry_point():
    import re
    decl = set(re.findall(r"^(?:int|void|const char\*) (fmt_[a-z0-9_]+)\(", open(os.path.join(REPO, "include", "fmt.h")).read(), re.M))
    src = open(os.path.join(SRC, "fmt_stub.cpp")).read()
    defined = set(re.findall(r"^(?:int|void|const char\*) (fmt_[a-z0-9_]+)\(", src, re.M))
    assert decl and decl == defined


def test_exit_driver_once(addon):
    rc, out, err = _run(addon)
    assert rc == 0, (out, err[-4000:])
    assert "exit-driver ok" in out and "AddressSanitizer" not in err


def test_exit_paths_200_runs_clean_under_asan(addon):
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        results = list(ex.map(lambda i: _run(addon, extra={"EXIT_ROUNDS": str(1 + i % 4)}), range(200)))
    bad = [(i, rc, err[-2000:]) for i, (rc, out, err) in enumerate(results)
           if rc != 0 or "exit-driver ok" not in out or "AddressSanitizer" in err]
    assert not bad, bad[:3]
