"""The one-process-per-stage pipeline (lvk_stage_step, what bench.py's layer-split
ranks run) with several processes on one GPU: every stage a child process (tests/stage_worker.py)
over the host shared-memory link (lvk_stage_connect_shm), bit-exact against the unsplit context.
It replaces the single-process llama_eval_internal (reference llama.cpp:927-1197); the RCCL form
of the same link needs one GPU per rank and is covered by test_gpu_split.py's single-rank test.
A stage given a bad token must fail its step and make every other stage fail too (no hang)."""
import os
import subprocess
import sys
import uuid

import numpy as np
import pytest

from stage_worker import PROMPT

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "stage_worker.py")


def _bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def _run_stages(path, S, mode, tmp_path, n_ctx=128, timeout=240):
    name = "/lvk_test_%d_%s" % (os.getpid(), uuid.uuid4().hex[:8])
    outs = [str(tmp_path / ("stage%d_%s.npz" % (s, mode))) for s in range(S)]
    env = dict(os.environ, LVK_STAGE_TIMEOUT_S="60")
    procs = [subprocess.Popen([sys.executable, WORKER, path, str(S), str(s), name, mode, outs[s], str(n_ctx)],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env) for s in range(S)]
    logs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=timeout)
            logs.append((p.returncode, o.decode(errors="replace"), e.decode(errors="replace")[-2000:]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        shm = "/dev/shm" + name
        if os.path.exists(shm):
            os.unlink(shm)
    for s, (rc, o, e) in enumerate(logs):
        assert rc == 0 and ("STAGE-%d-DONE" % s) in o, "stage %d rc %d\n%s\n%s" % (s, rc, o, e)
    return [dict(np.load(f)) for f in outs]


def _reference(lvk, path, n_ctx=128):
    m = lvk.Llama(path, n_ctx=n_ctx)
    lg = m.eval(PROMPT, 0)[-1].copy()
    toks, tok = [], 1000
    for i in range(10):
        tok = m.eval_greedy(tok, len(PROMPT) + i)
        toks.append(tok)
    m.close()
    return lg, toks


@pytest.mark.gpu
@pytest.mark.parametrize("S", [2, 3])
def test_stage_processes_match_single_context(tiny_models, gpu_available, tmp_path, S):
    """tiny Q4_0 (32 layers) as S stage processes on one GPU: prompt in 4-token micro-batches
    and 10 greedy steps relayed last -> first equal the unsplit context bit for bit"""
    import lvk
    path = tiny_models["tiny_q4_0"]
    want_lg, want_toks = _reference(lvk, path)
    res = _run_stages(path, S, "run", tmp_path)
    assert np.array_equal(_bits(res[-1]["prompt_logits"]), _bits(want_lg))
    assert list(res[0]["tokens"]) == want_toks
    assert list(res[-1]["tokens"]) == want_toks
    assert all(r["failed_at"] == -1 for r in res)
    # the link probe (lvk_stage_link_probe) ran on every stage and left the link usable: the
    # next greedy step's token reached stage 0 from the last stage
    assert all(0.0 < float(r["hop_us"]) < 1e6 for r in res)
    assert int(res[0]["post_probe_token"]) == int(res[-1]["post_probe_token"])


@pytest.mark.gpu
def test_stage_processes_7b_shaped(model_dir, gpu_available, tmp_path):
    """2 stage processes of a 2-layer LLaMA-7B-shaped Q4_0 model (n_embd 4096: the decode
    matvecs of matvec_cu.hip run inside the stages)"""
    import lvk
    from oracle_lib import gen_model
    path = gen_model(os.path.join(model_dir, "w4096_l2.bin"), n_embd=4096, n_head=32, n_layer=2, ftype=2, seed=5)
    want_lg, want_toks = _reference(lvk, path)
    res = _run_stages(path, 2, "run", tmp_path)
    assert np.array_equal(_bits(res[-1]["prompt_logits"]), _bits(want_lg))
    assert list(res[0]["tokens"]) == want_toks


@pytest.mark.gpu
def test_stage_bad_token_fails_every_stage(tiny_models, gpu_available, tmp_path):
    """stage 0 gets an out-of-range token at greedy step 3: it fails that step before any
    transfer, aborts the link, and the other stages' step 3 fails too -- promptly, not at the
    60 s link time limit"""
    res = _run_stages(tiny_models["tiny_q4_0"], 3, "badtoken", tmp_path)
    for r in res:
        assert int(r["failed_at"]) == 3, [int(x["failed_at"]) for x in res]
        assert float(r["fail_s"]) < 30.0


@pytest.mark.gpu
def test_stage_link_reconnects_after_abort(tiny_models, gpu_available, tmp_path):
    """after the aborted step 3 every stage reconnects under the SAME shm name (stage 0 makes
    a fresh ring: no stale abort word, join count or messages) and redoes the step: the
    greedy stream equals the unsplit context's"""
    import lvk
    path = tiny_models["tiny_q4_0"]
    _, want_toks = _reference(lvk, path)
    res = _run_stages(path, 3, "reconnect", tmp_path)
    for r in res:
        assert int(r["failed_at"]) == 3
    assert list(res[0]["tokens"]) == want_toks
    assert list(res[-1]["tokens"]) == want_toks
