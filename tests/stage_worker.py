"""One pipeline stage in its own process (tests/test_gpu_stagelink.py): the C++ stage link
(lvk_stage_connect_shm + lvk_stage_step) exactly as a bench.py layer-split rank runs it, over
the host shared-memory ring instead of RCCL so that several stages can share one GPU.

usage: stage_worker.py <model> <n_stages> <stage> <shm name> <mode> <out.npz> [n_ctx]
  mode run      : prompt in micro-batches, then greedy steps; the last stage saves the
                  prompt logits, every greedy token is saved by stages 0 and S-1
  mode badtoken : like run, but stage 0 passes an out-of-range token at greedy step 3;
                  every stage must fail that step (none may hang)
  mode reconnect: like badtoken, then every stage reconnects under the same shm name and
                  redoes step 3 with the right token: the stream must be run's
No torch in this process (lvk.py refuses to share a process with torch's HIP runtime).
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama.vk_amd"))
import lvk  # noqa: E402

PROMPT = [1, 450, 4996, 17354, 1701, 29889, 13, 1576, 22, 3, 99, 1234, 77]


def main():
    path, S, s, name, mode, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5], sys.argv[6]
    n_ctx = int(sys.argv[7]) if len(sys.argv) > 7 else 128
    hp = lvk.model_hparams(path)
    L = hp["n_layer"]
    st = lvk.Llama(path, n_ctx=n_ctx, layers=(s * L // S, (s + 1) * L // S))
    st.stage_connect_shm(name, S, s)
    res = {"stage": s}
    first, last = s == 0, s == S - 1
    st.stage_step(PROMPT if first else None, len(PROMPT), 0, micro=4)
    if last:
        res["prompt_logits"] = st.logits()[-1].copy()
    toks, tok, failed_at = [], 1000, -1
    t0 = time.time()
    for i in range(10):
        arg = tok
        if mode in ("badtoken", "reconnect") and first and i == 3:
            arg = hp["n_vocab"] + 5
        try:
            tok = st.stage_step([arg] if first else None, 1, len(PROMPT) + i, greedy=True)
        except RuntimeError:
            failed_at = i
            if mode != "reconnect":
                break
            st.stage_connect_shm(name, S, s)
            tok = st.stage_step([tok] if first else None, 1, len(PROMPT) + i, greedy=True)
        toks.append(tok)
    res["fail_s"] = time.time() - t0
    res["tokens"] = np.array(toks, np.int32)
    if mode == "run" and failed_at < 0:
        # the link alone (lvk_stage_link_probe), then one more greedy step over the same link
        res["hop_us"] = st.stage_link_probe(hp["n_embd"] * 4, 16)
        res["post_probe_token"] = st.stage_step([tok] if first else None, 1, len(PROMPT) + 10, greedy=True)
    res["failed_at"] = failed_at
    st.close()
    np.savez(out, **res)
    print("STAGE-%d-DONE" % s, flush=True)


if __name__ == "__main__":
    main()
