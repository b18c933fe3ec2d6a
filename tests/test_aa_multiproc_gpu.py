"""The multi-rank data path with real renders in two processes on the GPU
(tools/multiproc_gpu_check.py: tile sets gathered through rtmi.dist.FramePipeline, Expected
SARSA's TD all-reduce through rtmi.dist.sarsa_frame, over gloo with both ranks on cuda:0;
everything bit-exact against one process).  The file sorts first: the launcher is started
before this pytest process has touched the GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_two_process_tiles_and_td_exchange(tmp_path):
    out = tmp_path / "mp.json"
    # --standalone: the launcher's rendezvous store binds a free port itself (no probe race)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--standalone", "--local-addr", "127.0.0.1",
           os.path.join(ROOT, "tools", "multiproc_gpu_check.py"), "--out", str(out)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.exists(), (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    res = json.loads(out.read_text())
    assert res["render"]["ok"], res
    assert res["sarsa"]["ok"], res
    assert r.returncode == 0, r.stderr[-2000:]
