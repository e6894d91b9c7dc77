"""Layer-split pipeline host logic, world_size 2 and 3 over gloo on the CPU
(torch.distributed, in spawned worker processes: torch never enters the test process, which
loads the HIP library).  The real stages run the C++ stage link: tests/test_gpu_stagelink.py."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama.vk_amd"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_layer_ranges():
    from pipeline import layer_ranges
    for L in (2, 32, 40, 80):
        for S in (1, 2, 4, 8):
            if S > L:
                continue
            r = layer_ranges(L, S)
            assert r[0][0] == 0 and r[-1][1] == L
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
            assert max(e - b for b, e in r) - min(e - b for b, e in r) <= 1
    assert layer_ranges(80, 8) == [(10 * s, 10 * s + 10) for s in range(8)]
    with pytest.raises(ValueError):
        layer_ranges(2, 3)


class FakeStage:
    """numpy stand-in for an lvk stage: embeddings, per-layer affine maps, lm_head;
    f32 arithmetic so a split must reproduce the single-process bits"""
    E, V, L = 16, 50, 6

    def __init__(self, layers):
        rng = np.random.default_rng(0)
        self.emb = rng.standard_normal((self.V, self.E)).astype(np.float32)
        self.a = rng.standard_normal((self.L, self.E)).astype(np.float32)
        self.b = rng.standard_normal((self.L, self.E)).astype(np.float32)
        self.w = rng.standard_normal((self.E, self.V)).astype(np.float32)
        self.lb, self.le = layers
        self.x = np.zeros((64, self.E), np.float32)
        self.hist = []

    def stage_eval(self, tokens, n, n_past):
        if tokens is not None:
            self.x[:n] = self.emb[np.asarray(tokens)]
        for l in range(self.lb, self.le):
            self.x[:n] = np.tanh(self.x[:n] * self.a[l] + self.b[l] + np.float32(n_past) * np.float32(1e-3))
        self.n = n

    def get_x(self, ptr, n, on_device):
        import ctypes
        ctypes.memmove(ptr, self.x[:n].ctypes.data, n * self.E * 4)

    def set_x(self, ptr, n, on_device):
        import ctypes
        ctypes.memmove(self.x[:n].ctypes.data, ptr, n * self.E * 4)

    def logits(self):
        return (self.x[self.n - 1:self.n] @ self.w).astype(np.float32)


def _fake_worker(rank, world, port, q):
    import torch.distributed as dist
    from pipeline import StagePipeline, layer_ranges
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    st = FakeStage(layer_ranges(FakeStage.L, world)[rank])
    pipe = StagePipeline(st, FakeStage.E, 64, dist, on_device=False)
    out = pipe.decode([1, 7, 3], 10)
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_fake_pipeline_matches_single_process(world):
    import multiprocessing as mp   # the workers import torch; this (test) process must not
    ref = FakeStage((0, FakeStage.L))
    toks, n_past, out = [1, 7, 3], 0, []
    ref.stage_eval(toks, len(toks), n_past)
    n_past += len(toks)
    tok = int(np.argmax(ref.logits()[-1]))
    for _ in range(10):
        out.append(tok)
        ref.stage_eval([tok], 1, n_past)
        n_past += 1
        tok = int(np.argmax(ref.logits()[-1]))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fake_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(res[r] == out for r in range(world))
