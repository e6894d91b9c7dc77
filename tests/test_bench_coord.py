"""bench.py's N > 1 process layout on the CPU (world_size 2 and 3 over gloo, torchrun):
every rank's parent holds the gloo group and never loads the HIP library; the GPU work runs in
a worker child that never imports torch and reaches its peers through the parent (barrier,
max over ranks, broadcast from rank 0); rank 0's parent prints the one JSON line."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("ws", [2, 3])
def test_bench_worker_coordination(ws):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ws),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(ws), "--coord-selftest"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["ws"] == ws and out["rank"] == 0
    assert out["max"] == float(ws)
    assert out["bcast"] == {"uid": "ab" * 64}
    assert out["gather"] == [{"r": r} for r in range(ws)]
    assert out["torch_in_worker"] is False
