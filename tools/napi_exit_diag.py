"""Diagnostics (GPU box): runs the JS V1 merge-info replay of tests/test_napi.py a few times under
node with FMT_NAPI_BACKTRACE=1, printing each exit code and any native stack a SIGSEGV printed."""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), ROOT]
from test_napi import _v1_reload_js  # noqa: E402
from test_snapshot_v1 import v1_reload_inputs  # noqa: E402

import oracle  # noqa: E402  (the checker builds the inputs, as in the test)

oracle.build()
cases = v1_reload_inputs()
close = "e.close();" if "--no-close" not in sys.argv else ""
js = ("(async()=>{" + _v1_reload_js(cases) + "const e=new fmt.Engine(0);const r=await e.replayMergeTree(b.finish());"
      f"const t=[];for(let i=0;i<{len(cases)};i++) t.push(r.getText(i));{close}"
      "process.stdout.write(JSON.stringify(t).length+'\\n');})().catch((e)=>{console.error(e);process.exit(1);});")
with tempfile.NamedTemporaryFile("w", suffix=".js", delete=False) as f:
    f.write(js)
env = dict(os.environ, FMT_NAPI_BACKTRACE="1")
for i in range(int(os.environ.get("DIAG_RUNS", "3"))):
    r = subprocess.run(["node", f.name], capture_output=True, text=True, timeout=120, env=env)
    print(f"run {i}: rc={r.returncode} stdout={r.stdout.strip()[:80]}", flush=True)
    if r.stderr:
        print(r.stderr[-4000:], flush=True)
