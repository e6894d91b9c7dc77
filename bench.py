#!/usr/bin/env python3
"""bench.py -- LLaMA-7B Q4_0 single-stream decode on MI355X (BASELINE.json configs[1]).

A step = one llama_eval of one token (the reference main's greedy loop:
llama_eval -> argmax of the returned logits -> next token), on a seeded
synthetic 7B Q4_0 ggjt file (no checkpoints exist here).  Workload: 16-token
prompt, the context window filled once (positions 16..511, untimed), then K
timed greedy decode steps at positions spread evenly over 16..511 of the n_ctx
512 window (K = 496: every position in order; K > 496 wraps), so the rate is
the whole window's average whatever K is (the decode attention's cost grows
with the position).  Weights and KV cache are resident in HBM before the timed
region.

Also reported on the same line:
  prompt_eval   one 512-token llama_eval (BASELINE.json configs[2]), best of 3
  roofline      dominant kernel's algorithmic weight bytes per launch / its
                average duration, HIP events on the launch stream (profiled
                decode pass right after the timed region)
  cpu_baseline  the reference AVX2 ggml.c build (oracle/_ref, compiled from
                /root/reference) on the same file, host cores, bounded sample

Multi-GPU (torchrun): the 7B model does not shard: every rank
runs an independent replica; value = total tokens of all ranks / max time.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "llama.vk_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
MODEL_BYTES_7B = 4130490880    # algorithmic weight bytes per token
MODEL_BYTES_13B_Q41 = 9640369920   # 13B Q4_1 weight bytes per token
MODEL_BYTES_65B = 40644154368  # 65B Q4_0 weight bytes per token
CFG_65B = dict(n_embd=8192, n_head=64, n_layer=80, ftype=2, seed=3)
REF_PUBLISHED_TOKS = 16.3      # 7B Q4_0 predict 61.41 ms/token
LAYER_MAT_WEIGHTS_7B = 32 * (4 * 4096 * 4096 + 3 * 4096 * 11008)   # weights of the 7B layer matrices
VALU_FP32_TFLOPS = 157.3       # MI355X_MICROARCH.md: peak FP32 vector
INT8_DENSE_TOPS = 5000.0       # dense INT8/FP8 matrix-core peak (no 2:1 sparsity)


def prompt_tokens(n):
    return [1] + [100 + (i * 7919) % 31000 for i in range(1, n)]


class _StdoutToStderr:
    """gloo prints connection notices on fd 1; the driver reads one JSON line there"""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *a):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


class LocalCoord:
    """N = 1: no peers"""
    rank, ws, local = 0, 1, 0

    def barrier(self):
        pass

    def max(self, v):
        return v

    def bcast(self, obj):
        return obj

    def gather(self, obj):
        return [obj]


class PipeCoord:
    """N > 1, in the worker process: the barrier, max over ranks and broadcast from rank 0 are
    asked of the parent (which holds the gloo group) over a pipe.  The worker imports lvk and
    never torch; the parent imports torch and never lvk: one HIP runtime per process
    (profiles/r03_runtime_mix.md)."""

    def __init__(self, rfd, wfd):
        self.r = os.fdopen(rfd, "r")
        self.w = os.fdopen(wfd, "w")
        self.ws = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))

    def _ask(self, op, v=None):
        self.w.write(json.dumps({"op": op, "v": v}) + "\n")
        self.w.flush()
        line = self.r.readline()
        if not line:
            raise SystemExit("bench worker: parent closed the coordination pipe")
        return json.loads(line)["v"]

    def barrier(self):
        self._ask("barrier")

    def max(self, v):
        return float(self._ask("max", v))

    def bcast(self, obj):
        return self._ask("bcast", obj)

    def gather(self, obj):
        """every rank's obj, in rank order, on every rank"""
        return self._ask("gather", obj)

    def result(self, obj):
        self._ask("result", obj)


def serve_worker(argv):
    """N > 1 parent (one per rank under torchrun): joins the gloo group, runs the GPU work in a
    worker child (bench.py --worker) and answers its barrier / max / broadcast requests; rank 0
    prints the JSON line the worker hands back.  Returns the worker's exit code."""
    import datetime
    import torch.distributed as dist
    ws = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    with _StdoutToStderr():
        dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=20))
    p2c_r, p2c_w = os.pipe()
    c2p_r, c2p_w = os.pipe()
    env = dict(os.environ, LVK_BENCH_FDS="%d,%d" % (p2c_r, c2p_w))
    child = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--worker"] + argv,
                             pass_fds=(p2c_r, c2p_w), env=env, stdout=sys.stderr)
    os.close(p2c_r)
    os.close(c2p_w)
    rd, wr = os.fdopen(c2p_r, "r"), os.fdopen(p2c_w, "w")
    result = None
    import torch
    while True:
        line = rd.readline()
        if not line:
            break
        msg = json.loads(line)
        op, v = msg["op"], msg["v"]
        if op == "barrier":
            dist.barrier()
        elif op == "max":
            t = torch.tensor([float(v)], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            v = float(t.item())
        elif op == "bcast":
            box = [v]
            dist.broadcast_object_list(box, src=0)
            v = box[0]
        elif op == "gather":
            out = [None] * ws
            dist.all_gather_object(out, v)
            v = out
        elif op == "result":
            result = v
        wr.write(json.dumps({"v": v}) + "\n")
        wr.flush()
    rc = child.wait()
    if rank == 0 and result is not None:
        print(json.dumps(result), flush=True)
    dist.destroy_process_group()
    return rc if result is not None or rank != 0 else (rc or 1)


def ensure_model(path, coord, cfg):
    if coord.rank == 0 and not os.path.exists(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        import lvk
        tmp = path + ".tmp"
        lvk.gen_model(tmp, vocab=os.path.join(ROOT, "tests", "golden", "vocab32000.bin"), **cfg)
        os.replace(tmp, path)
    coord.barrier()


def cpu_quota():
    """CPUs this process may use per the cgroup CPU controller (v2 cpu.max, v1
    cpu.cfs_quota_us / cpu.cfs_period_us): (cpus or None when unlimited, where it was read)"""
    try:
        lines = open("/proc/self/cgroup").read().splitlines()
    except OSError:
        return None, "no /proc/self/cgroup"
    for ln in lines:
        parts = ln.split(":", 2)
        if len(parts) != 3:
            continue
        hier, ctrls, path = parts
        cands = []
        if hier == "0" and ctrls == "":
            cands = [("/sys/fs/cgroup" + path.rstrip("/") + "/cpu.max", "v2"), ("/sys/fs/cgroup/cpu.max", "v2")]
        elif "cpu" in ctrls.split(","):
            for root in ("/sys/fs/cgroup/cpu,cpuacct", "/sys/fs/cgroup/cpu"):
                cands.append((root + path.rstrip("/") + "/cpu.cfs_quota_us", "v1"))
                cands.append((root + "/cpu.cfs_quota_us", "v1"))
        for f, kind in cands:
            try:
                if kind == "v2":
                    q, per = open(f).read().split()[:2]
                    return (None if q == "max" else float(q) / float(per)), f
                q = int(open(f).read())
                per = int(open(f.replace("cfs_quota_us", "cfs_period_us")).read())
                return (None if q < 0 else q / per), f
            except (OSError, ValueError):
                continue
    return None, "no cpu controller limit found"


def cpu_info():
    """host CPU facts for the baseline line: nproc, model, AVX flags,
    physical cores of this process's CPU set, the cgroup CPU quota"""
    info = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
    q, src = cpu_quota()
    info["cgroup_cpu_quota"] = q
    info["cgroup_cpu_quota_source"] = src
    try:
        txt = open("/proc/cpuinfo").read()
        for line in txt.splitlines():
            if line.startswith("model name"):
                info["model"] = line.split(":", 1)[1].strip()
                break
        flags = next((l.split(":", 1)[1].split() for l in txt.splitlines() if l.startswith("flags")), [])
        info["simd"] = [f for f in ("avx", "avx2", "fma", "f16c", "avx512f", "avx512bw") if f in flags]
    except OSError:
        pass
    try:
        out = subprocess.run(["lscpu", "-p=CPU,CORE,SOCKET"], capture_output=True, text=True, timeout=10).stdout
        aff = os.sched_getaffinity(0)
        cores = {(l.split(",")[2], l.split(",")[1]) for l in out.splitlines()
                 if l and not l.startswith("#") and int(l.split(",")[0]) in aff}
        info["physical_cores"] = len(cores)
    except Exception:
        info["physical_cores"] = None
    return info


def cpu_baseline(path, budget_s=20.0, label="7B Q4_0", prompt=True, seg_steps=16, n_seg=3):
    """The reference AVX2 ggml.c build (oracle/_ref/libref.so) on the same file and tokens:
    decode tok/s, best of n_seg segments, at two thread counts -- the usable cores (the
    physical cores of this process's CPU set, capped by the cgroup CPU quota) and the box's
    per-GPU share (OMP_NUM_THREADS, 16) -- each with its own half of the budget; value = the
    faster, and (prompt=True) the 512-token prompt batch at that thread count, best of 3 --
    llama.cpp:1186-1195's n_eval / t_eval and n_p_eval / t_p_eval."""
    from oracle_lib import REF_SO, Ref
    if not os.path.exists(REF_SO):
        return None
    import numpy as np
    info = cpu_info()
    share = int(os.environ.get("OMP_NUM_THREADS") or 0) or 16
    phys = info.get("physical_cores") or info["affinity"]
    usable = phys
    if info.get("cgroup_cpu_quota"):
        usable = max(1, min(phys, int(info["cgroup_cpu_quota"])))
    tried = sorted({max(1, usable), max(1, min(share, usable))}, reverse=True)
    ref = Ref()
    t_load = time.perf_counter()
    m = ref.model(path, 512)
    t_load = time.perf_counter() - t_load
    toks = np.array(prompt_tokens(16), np.int32)
    # a 2-step probe per thread count: a count far slower than the best (an oversubscribed
    # quota the cgroup files do not show) is reported, not given segments
    probe = {}
    for threads in tried:
        lg = m.eval(toks, 0, n_threads=threads)
        tok = int(np.argmax(lg[-1]))
        t0 = time.perf_counter()
        for i in range(2):
            lg = m.eval(np.array([tok], np.int32), 16 + i, n_threads=threads)
            tok = int(np.argmax(lg[-1]))
        probe[threads] = 2 / (time.perf_counter() - t0)
    slow = [t for t in tried if probe[t] < max(probe.values()) / 3]
    tried = [t for t in tried if t not in slow]
    rates = {}
    per_threads = (budget_s * (0.6 if prompt else 1.0)) / len(tried)
    for threads in tried:
        lg = m.eval(toks, 0, n_threads=threads)
        tok, n_past = int(np.argmax(lg[-1])), 16
        segs, used = [], 0.0
        for k in range(n_seg):
            t0 = time.perf_counter()
            for _ in range(seg_steps):
                lg = m.eval(np.array([tok], np.int32), n_past, n_threads=threads)
                tok = int(np.argmax(lg[-1]))
                n_past = n_past + 1 if n_past + 1 < 512 else 16
            dt = time.perf_counter() - t0
            segs.append(seg_steps / dt)
            used += dt
            # a segment that would overrun this thread count's budget is not started
            if k + 1 < n_seg and used + dt > per_threads:
                break
        rates[threads] = segs
    best_t = max(rates, key=lambda t: max(rates[t]))
    p512 = np.array(prompt_tokens(512), np.int32)
    pr = []
    for _ in range(3 if prompt else 0):                      # 512-token prompt batch, best of 3
        t0 = time.perf_counter()
        m.eval(p512, 0, n_threads=best_t)
        pr.append(512 / (time.perf_counter() - t0))
        if sum(512 / r for r in pr) > budget_s * 0.4 and len(pr) < 3:
            break
    m.close()
    out = {"value": max(rates[best_t]), "unit": "tok/s", "cores": best_t, "kind": "reference",
           "sample": "reference ggml.c AVX2 build (oracle/_ref, compiled from the reference sources), the same "
                     "synthetic %s file and tokens, n_ctx 512, f16 KV: 16-token prompt, then up to %d segments of "
                     "%d greedy decode steps at each of -t %s (the usable cores: physical cores of the CPU set "
                     "capped by the cgroup quota; and the per-GPU share), each thread count with its own budget; "
                     "value = the best segment at the faster thread count (-t %d)%s"
                     % (label, n_seg, seg_steps, " and ".join(str(t) for t in tried), best_t,
                        "; prompt = one 512-token batch at -t %d, best of %d" % (best_t, len(pr)) if prompt else ""),
           "decode_tok_s_by_threads": {str(t): max(v) for t, v in rates.items()},
           "decode_segments_by_threads": {str(t): v for t, v in rates.items()},
           "decode_segments_tok_s": rates[best_t], "probe_tok_s_by_threads": {str(t): v for t, v in probe.items()},
           "dropped_slow_thread_counts": slow, "load_s": t_load, "host": info}
    if prompt:
        out["prompt_tok_s"] = max(pr)
        out["prompt_runs_tok_s"] = pr
    return out


SPLIT_TIMEOUT_S = 420
SPLIT_FIRST_TOKEN = 1000       # the greedy token the split's first decode step embeds
SPLIT_FORCED_STEPS = 16        # teacher-forced steps whose logits digests the split must reproduce
SPLIT_LINK_LAPS = 64           # laps of the link probe (per_hop_us)


def split_child(args):
    """one pipeline stage in a child process (bench.py --split-child): the C++ stage link
    (lvk_stage_connect / lvk_stage_step: ncclRecv -> this stage's layers -> ncclSend on the
    stage's stream, greedy token relayed from the last stage to the first; or the same over
    the host shared-memory ring, --split-transport shm, for stages sharing a GPU).  Prints
    one JSON line."""
    import numpy as np
    import lvk
    S, s = args.split_stages, args.split_stage
    lvk.set_device(args.split_device)
    hp = lvk.model_hparams(args.split_model)
    L = hp["n_layer"]
    lr = (s * L // S, (s + 1) * L // S)
    t0 = time.time()
    st = lvk.Llama(args.split_model, n_ctx=512, layers=lr)
    load_s = time.time() - t0
    if args.split_transport == "shm":
        st.stage_connect_shm(args.split_uid, S, s)
    else:
        st.stage_connect(bytes.fromhex(args.split_uid), S, s)
    ptoks = np.array(prompt_tokens(16), np.int32)
    first = s == 0
    st.stage_step(ptoks if first else None, 16, 0, micro=args.split_micro)
    # the last stage's prompt logits, as the bit pattern's digest (compared with one unsplit context)
    lhash = logits_digest(st.logits()[-1]) if s == S - 1 else None
    tok, n_past = SPLIT_FIRST_TOKEN, 16
    toks = []
    for _ in range(args.warmup):
        tok = st.stage_step(np.array([tok], np.int32) if first else None, 1, n_past, greedy=True)
        toks.append(tok)
        n_past += 1
    t0 = time.perf_counter()
    for _ in range(args.steps_split):
        tok = st.stage_step(np.array([tok], np.int32) if first else None, 1, n_past, greedy=True)
        toks.append(tok)
        n_past = n_past + 1 if n_past + 1 < 512 else 16
    dec = time.perf_counter() - t0
    # the link alone (lvk_stage_link_probe): one token's residual stream around the stage ring,
    # SURVEY.md 8d's per-hop time; every stage takes part
    hop_us = st.stage_link_probe(hp["n_embd"] * 4, SPLIT_LINK_LAPS)
    # a 512-token prompt through the pipeline, with and without micro-batches (every rank
    # times its own stage_step; the last stage's time is the pipeline's)
    p512 = np.array(prompt_tokens(512), np.int32)
    pre = {}
    for micro in (args.split_micro, 0):
        best = 1e30
        for _ in range(2):
            st.stage_step(np.array([tok], np.int32) if first else None, 1, 16, greedy=True)   # re-sync the stages
            t0 = time.perf_counter()
            st.stage_step(p512 if first else None, 512, 0, micro=micro)
            best = min(best, time.perf_counter() - t0)
        pre[micro] = best
    # teacher-forced check pass: the 16-token prompt again, then SPLIT_FORCED_STEPS seeded
    # non-repeating tokens one step at a time (no greedy relay); the last stage digests every
    # step's logits row (lvk_logits_digest), compared with one unsplit context by rank 0
    from oracle_lib import forced_tokens
    st.stage_step(ptoks if first else None, 16, 0, micro=args.split_micro)
    fdig = []
    for i, t in enumerate(forced_tokens(SPLIT_FORCED_STEPS)):
        st.stage_step(np.array([t], np.int32) if first else None, 1, 16 + i)
        if s == S - 1:
            fdig.append(lvk.logits_digest(st.logits()[-1]))
    st.close()
    print(json.dumps({"stage": s, "layers": list(lr), "load_s": load_s, "decode_s": dec, "hop_us": hop_us,
                      "prefill_s": pre[args.split_micro], "prefill_nomicro_s": pre[0],
                      "tokens": toks if first else None, "prompt_logits_digest": lhash,
                      "forced_digests": [str(d) for d in fdig] if s == S - 1 else None}), flush=True)


def logits_digest(row):
    import hashlib
    import numpy as np
    return hashlib.sha256(np.ascontiguousarray(row, np.float32).view(np.uint32).tobytes()).hexdigest()[:32]


def greedy_tokens_1gpu(path, n):
    """the same steps as a split's stages on one unsplit context: the greedy steps (16-token
    prompt, then SPLIT_FIRST_TOKEN at n_past 16, ...) whose tokens the split's stream must equal,
    the digest of the prompt's last logits row, and the per-step logits digests of the
    teacher-forced pass (oracle_lib.forced_tokens at n_past 16..)"""
    import numpy as np
    import lvk
    from oracle_lib import forced_tokens
    m = lvk.Llama(path, n_ctx=512)
    ptoks = np.array(prompt_tokens(16), np.int32)
    digest = logits_digest(m.eval(ptoks, 0)[-1])
    tok, out = SPLIT_FIRST_TOKEN, []
    for i in range(n):
        tok = m.eval_greedy(tok, 16 + i)
        out.append(tok)
    m.eval(ptoks, 0)
    fdig = [str(lvk.logits_digest(m.eval([int(t)], 16 + i)[-1])) for i, t in enumerate(forced_tokens(SPLIT_FORCED_STEPS))]
    m.close()
    return out, digest, fdig


def layer_split(args, coord):
    """N > 1: LLaMA-65B Q4_0 (BASELINE configs[4]) split by layers over the ws ranks, one
    stage per GPU, residual stream over RCCL send/recv (the C++ stage link; --split-transport
    shm: the host shared-memory ring, so that the ranks of a one-GPU rehearsal can share the
    device).  Each rank runs its stage in a child process under a time limit, so a transport
    failure costs this line, not the bench.  Rank 0 then replays the first --split-check
    greedy steps on one unsplit context: the split's tokens must be the same."""
    path = args.split_model or os.path.join(os.path.dirname(args.model), "llama-65b-q4_0.bin")
    rank, ws, local = coord.rank, coord.ws, coord.local
    ensure_model(path, coord, CFG_65B)
    import lvk
    # the communicator id (or the shm ring's name) is made here, in a process without torch
    if args.split_transport == "shm":
        uid = coord.bcast("/lvk_bench_%d_%s" % (os.getpid(), os.urandom(6).hex()) if rank == 0 else None)
    else:
        uid = coord.bcast(lvk.rccl_unique_id().hex() if rank == 0 else None)
    cmd = [sys.executable, os.path.abspath(__file__), "--split-child", "--split-stages", str(ws),
           "--split-stage", str(rank), "--split-device", str(local % lvk.device_count()), "--split-uid", uid,
           "--split-model", path, "--steps-split", str(args.steps_split), "--warmup", "4",
           "--split-micro", str(args.split_micro), "--split-transport", args.split_transport]
    res, err = None, None
    try:
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=SPLIT_TIMEOUT_S)
        if p.returncode == 0:
            res = json.loads(p.stdout.decode().strip().splitlines()[-1])
        else:
            err = "rank %d stage exited %d: %s" % (rank, p.returncode, p.stderr.decode(errors="replace")[-400:])
    except subprocess.TimeoutExpired:
        err = "rank %d stage timed out after %d s" % (rank, SPLIT_TIMEOUT_S)
    except Exception as e:                       # noqa: BLE001 -- reported in the line
        err = "rank %d: %r" % (rank, e)
    finally:
        if args.split_transport == "shm" and rank == 0 and os.path.exists("/dev/shm" + uid):
            os.unlink("/dev/shm" + uid)         # a stage that died before every stage joined
    ok = coord.max(0.0 if res is not None else 1.0) == 0.0
    if not ok:
        return {"error": err or "another rank's stage failed", "transport": args.split_transport}
    dec = coord.max(res["decode_s"])
    hop_us = coord.max(res["hop_us"])
    pre = coord.max(res["prefill_s"])
    pre0 = coord.max(res["prefill_nomicro_s"])
    digest_split = coord.gather(res.get("prompt_logits_digest"))[-1]     # the last stage's
    fdig_split = coord.gather(res.get("forced_digests"))[-1]
    check = None
    if rank == 0 and args.split_check > 0:
        n = min(args.split_check, len(res["tokens"]))
        t0 = time.time()
        want, digest, fdig = greedy_tokens_1gpu(path, n)
        check = {"n_tokens": n, "tokens_split": res["tokens"][:n], "tokens_1gpu": want,
                 "match": res["tokens"][:n] == want, "check_s": time.time() - t0,
                 "positions": "16..%d" % (16 + n - 1), "first_token": SPLIT_FIRST_TOKEN,
                 "prompt_logits_digest_split": digest_split, "prompt_logits_digest_1gpu": digest,
                 "prompt_logits_bit_identical": digest_split == digest,
                 "forced_steps": {"n": SPLIT_FORCED_STEPS, "positions": "16..%d" % (15 + SPLIT_FORCED_STEPS),
                                  "tokens": "oracle_lib.forced_tokens (seeded, non-repeating)",
                                  "digests_split": fdig_split, "digests_1gpu": fdig,
                                  "logits_bit_identical_every_step": fdig_split == fdig}}
    coord.barrier()
    L = CFG_65B["n_layer"]
    r = args.steps_split / dec
    hops = {"per_hop_us": hop_us, "message_bytes": CFG_65B["n_embd"] * 4, "laps": SPLIT_LINK_LAPS,
            "hops_per_token": ws,
            "method": "lvk_stage_link_probe: laps of one token's residual stream (n_embd f32) around the stage "
                      "ring on the stage link's transport and stream, wall time per lap over the stages (max "
                      "over ranks)"}
    transport = ("RCCL (ncclCommInitRank over the %d ranks)" % ws if args.split_transport == "rccl" else
                 "host shared-memory ring (lvk_stage_connect_shm; the one-GPU rehearsal of the RCCL link)")
    return {"value": r, "unit": "tok/s", "stages": ws, "steps": args.steps_split, "ms_per_token": 1e3 / r,
            "layers_per_stage": [[s * L // ws, (s + 1) * L // ws] for s in range(ws)],
            "workload": "LLaMA-65B Q4_0 (synthetic, seed 3) greedy decode, layers split over %d stages (one "
                        "stage per rank: recv -> layers -> send of inpL f32 [n_embd] on the stage stream, greedy "
                        "token relayed last -> first), n_ctx 512" % ws,
            "frac_hbm_roofline_1gpu": r * MODEL_BYTES_65B / 1e9 / HBM_PEAK_GBS,
            "prefill_512": {"tok_s": 512 / pre, "ms": pre * 1e3, "micro_batch": args.split_micro,
                            "tok_s_no_micro_batch": 512 / pre0},
            "link": hops,
            "transport": transport, "devices": "rank r on device LOCAL_RANK %% %d" % lvk.device_count(),
            "greedy_check": check}


def decode_65b(args, coord, n_ctx, ptoks):
    """LLaMA-65B Q4_0 single-stream decode on ONE GPU (BASELINE configs[4] at S = 1: the
    40.6 GB of weights fit in 288 GB of HBM): tok/s, fraction of the model-bytes roofline
    (197 tok/s at 8 TB/s) and a per-kernel-class profile"""
    import numpy as np
    import lvk
    path = os.path.join(os.path.dirname(args.model), "llama-65b-q4_0.bin")
    t0 = time.time()
    ensure_model(path, coord, CFG_65B)
    gen_s = time.time() - t0
    t0 = time.time()
    m = lvk.Llama(path, n_ctx=n_ctx)
    load_s = time.time() - t0
    # the window is filled once (every K / V row exists), then the timed steps are spread
    # evenly over positions 16..n_ctx-1, as in the 7B line
    tok = fill_window(m, ptoks, n_ctx)
    coord.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps_65b):
        tok = int(np.argmax(m.eval([tok], spread_pos(i, args.steps_65b, n_ctx), copy=False)[-1]))
    dt = coord.max(time.perf_counter() - t0)
    r = args.steps_65b / dt
    m.set_profiling(True)
    m.reset_profile()
    for i in range(8):
        tok = int(np.argmax(m.eval([tok], 16 + i * 60)[-1]))
    prof = m.profile()
    m.set_profiling(False)
    # teacher-forced stream check (a synthetic model's greedy stream repeats one token): the
    # chained device decode must reproduce every per-step llama_eval logits digest
    stream = stream_check(m, ptoks, args.stream_check_65b)
    # 1-GPU 65B 512-token prompt (best of 2): the S = 1 reference point of the split's prefill
    ptoks512 = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, n_ctx)], np.int32)
    best = 1e30
    for _ in range(2):
        coord.barrier()
        t0 = time.perf_counter()
        m.eval(ptoks512, 0)
        best = min(best, coord.max(time.perf_counter() - t0))
    prompt_image = m.prompt_image_bytes()
    m.close()
    cpu65 = None
    if coord.rank == 0 and coord.ws == 1 and not args.no_cpu_baseline:
        # the reference on the same 40.6 GB file: a few decode steps
        cpu65 = cpu_baseline(path, args.cpu_budget, label="65B Q4_0", prompt=False, seg_steps=2, n_seg=2)
    fmas = 80 * (4 * 8192 * 8192 + 3 * 8192 * 22016) / 4 * len(ptoks512)
    prompt = {"value": len(ptoks512) / best, "unit": "tok/s", "n_tokens": len(ptoks512), "ms": best * 1e3,
              "a16_image_bytes": prompt_image,
              "roofline": {"bound": "valu-fp32 (the reference's sequential fp32 FMA chains)",
                           "achieved": 2 * fmas / best / 1e12, "peak": VALU_FP32_TFLOPS, "unit": "TFLOP/s",
                           "frac": 2 * fmas / best / 1e12 / VALU_FP32_TFLOPS, "fp32_chain_fmas": fmas}}
    kernels = {k: {"avg_us": v["ms"] / v["launches"] * 1e3,
                   "gbs": (v["bytes"] / v["launches"]) / (v["ms"] / v["launches"] * 1e-3) / 1e9 if v["bytes"] else None}
               for k, v in prof.items() if v["launches"]}
    return {"value": r, "unit": "tok/s", "steps": args.steps_65b, "ms_per_token": 1e3 / r, "prompt_eval": prompt,
            "workload": "LLaMA-65B Q4_0 (synthetic, seed 3; n_embd 8192, 64 heads, 80 layers, n_ff 22016) "
                        "single-stream greedy decode on 1 GPU, %d steps at positions spread evenly over "
                        "16..%d (window filled first), n_ctx %d" % (args.steps_65b, n_ctx - 1, n_ctx),
            "model_bytes_per_token": MODEL_BYTES_65B,
            "frac_hbm_roofline": r * MODEL_BYTES_65B / 1e9 / HBM_PEAK_GBS,
            "roofline_tok_s": HBM_PEAK_GBS * 1e9 / MODEL_BYTES_65B,
            "kernels": kernels, "gen_s": gen_s, "load_s": load_s, "cpu_baseline": cpu65,
            "stream_check": stream,
            "vs_cpu_baseline": (r / cpu65["value"]) if cpu65 else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--steps", type=int, default=496)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--model", default="/tmp/lvk_bench/llama-7b-q4_0.bin")
    ap.add_argument("--prompt-evals", type=int, default=3)
    ap.add_argument("--profile-steps", type=int, default=48)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-greedy", action="store_true",
                    help="skip the lvk_eval_greedy decode leg")
    ap.add_argument("--no-13b", action="store_true", help="skip the 13B Q4_1 decode line (BASELINE configs[3])")
    ap.add_argument("--steps-13b", type=int, default=96)
    ap.add_argument("--no-65b", action="store_true", help="skip the 1-GPU 65B decode line (BASELINE configs[4], S=1)")
    ap.add_argument("--steps-65b", type=int, default=32)
    ap.add_argument("--no-split", action="store_true", help="N>1: skip the layer-split pipeline line (SURVEY 8e)")
    ap.add_argument("--steps-split", type=int, default=48)
    ap.add_argument("--split-model", default=None, help="model for the layer-split line (default: the 65B file)")
    ap.add_argument("--split-micro", type=int, default=64, help="prompt micro-batch of the layer split (tokens)")
    ap.add_argument("--split-transport", choices=("rccl", "shm"), default="rccl",
                    help="stage link of the layer split: RCCL (one GPU per rank, the default) or the host "
                         "shared-memory ring (ranks may share a GPU: the one-GPU rehearsal)")
    ap.add_argument("--stream-check", type=int, default=64,
                    help="teacher-forced steps whose per-step logits digests the chained path must reproduce")
    ap.add_argument("--stream-check-13b", type=int, default=32)
    ap.add_argument("--stream-check-65b", type=int, default=16)
    ap.add_argument("--split-check", type=int, default=16,
                    help="greedy steps of the split replayed on one unsplit context by rank 0 (0: none)")
    ap.add_argument("--split-rehearse", action="store_true",
                    help="run the layer-split leg at N = 1 too (one stage: the RCCL link on one rank)")
    ap.add_argument("--worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--coord-selftest", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--split-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--split-stages", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--split-stage", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--split-device", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--split-uid", default="", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r06_traffic.json"))
    args = ap.parse_args()
    if args.split_child:
        split_child(args)
        return
    if args.worker:
        rfd, wfd = (int(x) for x in os.environ["LVK_BENCH_FDS"].split(","))
        coord = PipeCoord(rfd, wfd)
        coord.result(run(args, coord))
        return
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        sys.exit(serve_worker(sys.argv[1:]))
    out = run(args, LocalCoord())
    print(json.dumps(out))
    if out and not out.get("checks", {}).get("passed", True):
        sys.stderr.write("bench: correctness checks failed: %s\n" % out["checks"]["failed"])
        sys.exit(1)


def run(args, coord):
    """every leg of the bench on this rank's GPU; returns rank 0's JSON object (None elsewhere)"""
    ws, rank, local = coord.ws, coord.rank, coord.local
    if args.coord_selftest:
        # the N > 1 plumbing without a GPU (tests/test_bench_coord.py): no lvk, no torch here
        coord.barrier()
        mx = coord.max(float(rank + 1))
        b = coord.bcast({"uid": "ab" * 64} if rank == 0 else None)
        g = coord.gather({"r": rank})
        coord.barrier()
        return {"ws": ws, "rank": rank, "max": mx, "bcast": b, "gather": g, "torch_in_worker": "torch" in sys.modules} \
            if rank == 0 else None
    n_gpus = args.gpus if args.gpus else ws
    import numpy as np
    import lvk
    if lvk.device_count() < 1:
        raise SystemExit("bench: no GPU visible")
    if ws > 1:
        lvk.set_device(local % lvk.device_count())
    cfg = dict(n_embd=4096, n_head=32, n_layer=32, ftype=2, seed=1)
    ensure_model(args.model, coord, cfg)

    t0 = time.time()
    m = lvk.Llama(args.model, n_ctx=512)
    load_s = time.time() - t0
    n_ctx = 512
    ptoks = np.array(prompt_tokens(16), np.int32)

    # warmup: prompt + W decode steps (also instantiates the decode graph), then the window is
    # filled once (every position's K / V rows exist before a timed step reads them)
    lg = m.eval(ptoks, 0)
    tok, n_past = int(np.argmax(lg[-1])), 16
    for i in range(args.warmup):
        lg = m.eval([tok], 16 + (i % (n_ctx - 16)))
        tok = int(np.argmax(lg[-1]))
    lg = m.eval(ptoks, 0)
    tok = int(np.argmax(lg[-1]))
    for p in range(16, n_ctx):
        tok = int(np.argmax(m.eval([tok], p)[-1]))
    win = n_ctx - 16

    def pos_of(i):
        # K <= 496: positions spread evenly over 16..511 (K = 496: each once, in order)
        return 16 + (i * win // args.steps if args.steps <= win else i % win)

    # timed region: K greedy decode steps
    lg = m.eval(ptoks, 0)
    tok = int(np.argmax(lg[-1]))
    coord.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        # llama_eval + argmax over llama_get_logits' row, as examples/main reads it (no copy)
        lg = m.eval([tok], pos_of(i), copy=False)
        tok = int(np.argmax(lg[-1]))
    t1 = time.perf_counter()
    coord.barrier()
    elapsed = coord.max(t1 - t0)
    value = n_gpus * args.steps / elapsed
    positions = ("16..511, each once in order" if args.steps == win else
                 "spread evenly over 16..511 (window filled first)" if args.steps < win else
                 "16..511 wrapping to 16 after 511")

    greedy = None
    if not args.no_greedy:
        # same decode with the sampler on the device (lvk_eval_greedy): the
        # argmax runs over the logits in HBM and 4 bytes come back instead of 128 KB
        m.eval(ptoks, 0)
        tok = int(np.argmax(m.logits()[-1]))
        tok_first = tok
        seq_g = []
        coord.barrier()
        t0 = time.perf_counter()
        for i in range(args.steps):
            tok = m.eval_greedy(tok, 16 + (i % (n_ctx - 16)))
            seq_g.append(tok)
        t1 = time.perf_counter()
        coord.barrier()
        el_g = coord.max(t1 - t0)
        greedy = {"value": n_gpus * args.steps / el_g, "unit": "tok/s", "ms_per_step": el_g / args.steps * 1e3,
                  "path": "lvk_eval_greedy: decode graph ending in the device argmax, 4-byte D2H",
                  "first_token": tok_first}
        # the same greedy steps chained on the device (lvk_decode_greedy): one call per pass
        # over positions 16..n_ctx-1, the step graph replayed back to back; its tokens must be
        # the per-step loop's
        m.eval(ptoks, 0)
        seq_c = []
        coord.barrier()
        t0 = time.perf_counter()
        tok, i = tok_first, 0
        while i < args.steps:
            pos = 16 + (i % (n_ctx - 16))
            n = min(args.steps - i, n_ctx - pos)
            part = m.decode_greedy(tok, pos, n)
            seq_c.extend(int(t) for t in part)
            tok, i = int(part[-1]), i + n
        t1 = time.perf_counter()
        coord.barrier()
        el_c = coord.max(t1 - t0)
        greedy["chained"] = {"value": n_gpus * args.steps / el_c, "unit": "tok/s", "ms_per_step": el_c / args.steps * 1e3,
                             "path": "lvk_decode_greedy: one call per pass over positions 16..511, the step graph "
                                     "replayed back to back (argmax, step block and next embedding row on the device)",
                             "tokens_match_eval_greedy": seq_c == seq_g}
        # teacher-forced stream check (a synthetic model's greedy stream settles on one token, so
        # the check above passes under many numeric errors): seeded non-repeating tokens through
        # per-step llama_eval and through lvk_decode_chain; every step's device logits digest must
        # equal the digest of the per-step logits row
        greedy["stream_check"] = stream_check(m, ptoks, args.stream_check)
        # host sampler (llama_sample_top_p_top_k, main's defaults: top_k 40, top_p 0.95, temp 0.8,
        # repeat_penalty 1.1 over a 64-token window) on fresh logits (lvk_eval_greedy leaves none)
        m.eval([tok], 16)
        last64 = np.array(prompt_tokens(64), np.int32)
        t0 = time.perf_counter()
        for _ in range(200):
            m.sample(last64, 40, 0.95, 0.8, 1.1)
        greedy["host_sampler_us"] = (time.perf_counter() - t0) / 200 * 1e6
        # sampled decode at main's defaults: llama_eval + the host sampler over all logits,
        # against lvk_eval_sample (repeat penalty, temperature and top-k on the device, the
        # host finishing over the 40 candidates)
        rates = {}
        for mode in ("host", "device"):
            m.eval(ptoks, 0)
            win = list(prompt_tokens(64))
            tok = m.sample(np.array(win, np.int32), 40, 0.95, 0.8, 1.1)
            t0 = time.perf_counter()
            for i in range(args.steps):
                win = win[1:] + [tok]
                pos = 16 + (i % (n_ctx - 16))
                if mode == "host":
                    m.eval([tok], pos)
                    tok = m.sample(np.array(win, np.int32), 40, 0.95, 0.8, 1.1)
                else:
                    tok = m.eval_sample(tok, pos, np.array(win, np.int32), 40, 0.95, 0.8, 1.1)
            rates[mode] = args.steps / (time.perf_counter() - t0)
        greedy["sampled_decode_tok_s"] = {"host_sampler": rates["host"], "device_sampler": rates["device"],
                                          "settings": "top_k 40, top_p 0.95, temp 0.8, repeat_penalty 1.1 over 64"}

    # prompt eval: one 512-token batch (configs[2])
    p512 = np.array(prompt_tokens(512), np.int32)
    best = 1e30
    for _ in range(args.prompt_evals):
        t0 = time.perf_counter()
        m.eval(p512, 0)
        best = min(best, time.perf_counter() - t0)
    best = coord.max(best)
    # the bit-faithful floor is the reference's fp32 chains -- one fmaf per
    # 4-element integer partial -- at the VALU FP32 peak; the INT8 line prices the same
    # matmul MACs on the dense matrix-core peak (what a non-faithful GEMM could reach)
    fmas = 512 * LAYER_MAT_WEIGHTS_7B / 4
    macs = 512 * LAYER_MAT_WEIGHTS_7B
    prompt = {"value": n_gpus * 512 / best, "unit": "tok/s", "n_tokens": 512, "ms": best * 1e3,
              "a16_image_bytes": m.prompt_image_bytes(),
              "path": "matrix cores (v_mfma_f32_32x32x8_f16 exact 4-element integer partials, f32 MFMA scale "
                      "products) + VALU fp32 chains; bit-identical to the AVX2 reference",
              "roofline": {"bound": "valu-fp32 (the reference's sequential fp32 FMA chains)",
                           "achieved": 2 * fmas / best / 1e12, "peak": VALU_FP32_TFLOPS, "unit": "TFLOP/s",
                           "frac": 2 * fmas / best / 1e12 / VALU_FP32_TFLOPS, "fp32_chain_fmas": fmas},
              "int8_mfma_equiv": {"ops": 2 * macs, "achieved_tops": 2 * macs / best / 1e12,
                                  "peak_tops": INT8_DENSE_TOPS, "frac": 2 * macs / best / 1e12 / INT8_DENSE_TOPS}}
    m.set_profiling(True)
    m.reset_profile()
    m.eval(p512, 0)
    pp = m.profile()
    m.set_profiling(False)
    prompt["kernels_ms"] = {k: v["ms"] for k, v in pp.items() if v["launches"]}

    # profiled decode pass: HIP events around every kernel class
    m.set_profiling(True)
    m.reset_profile()
    lg = m.eval(ptoks, 0)
    m.reset_profile()
    tok = int(np.argmax(lg[-1]))
    for i in range(args.profile_steps):
        lg = m.eval([tok], 16 + i * (n_ctx - 17) // max(1, args.profile_steps))
        tok = int(np.argmax(lg[-1]))
    prof = m.profile()
    m.set_profiling(False)
    kernels = {}
    for k, v in prof.items():
        if v["launches"]:
            avg = v["ms"] / v["launches"]
            kernels[k] = {"avg_us": avg * 1e3, "ms_per_token": v["ms"] / args.profile_steps,
                          "gbs": (v["bytes"] / v["launches"]) / (avg * 1e-3) / 1e9 if v["bytes"] else None}
    dom = max((k for k in kernels if prof[k]["bytes"]), key=lambda k: prof[k]["ms"])
    bpl = prof[dom]["bytes"] / prof[dom]["launches"]
    avg_s = prof[dom]["ms"] / prof[dom]["launches"] * 1e-3
    traffic = None
    if not os.path.exists(args.traffic_json):     # the previous round's record
        args.traffic_json = os.path.join(ROOT, "profiles", "r04_traffic.json")
    if os.path.exists(args.traffic_json):
        try:
            traffic = json.load(open(args.traffic_json)).get(dom, {}).get("bytes_per_launch")
        except Exception:
            traffic = None
    achieved = bpl / avg_s / 1e9
    roofline = {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "bytes_per_launch": bpl,
                "avg_launch_us": avg_s * 1e6}
    step_gbs = value / n_gpus * MODEL_BYTES_7B / 1e9

    # 13B Q4_1 single-stream decode (BASELINE.json configs[3]), same loop
    m.close()          # one model resident at a time from here on
    q41 = None
    if not args.no_13b:
        path13 = os.path.join(os.path.dirname(args.model), "llama-13b-q4_1.bin")
        ensure_model(path13, coord, dict(n_embd=5120, n_head=40, n_layer=40, ftype=3, seed=2))
        m13 = lvk.Llama(path13, n_ctx=n_ctx)
        tok = fill_window(m13, ptoks, n_ctx)
        coord.barrier()
        t0 = time.perf_counter()
        for i in range(args.steps_13b):
            lg = m13.eval([tok], spread_pos(i, args.steps_13b, n_ctx), copy=False)
            tok = int(np.argmax(lg[-1]))
        t13 = coord.max(time.perf_counter() - t0)
        stream13 = stream_check(m13, ptoks, args.stream_check_13b)
        image13 = m13.prompt_image_bytes()
        # per-kernel-class HIP-event pass (the Q4_1 decode kernels, matvec_cu41.hip)
        m13.set_profiling(True)
        m13.reset_profile()
        for i in range(16):
            lg = m13.eval([tok], 16 + i * 31)
            tok = int(np.argmax(lg[-1]))
        p13 = m13.profile()
        m13.set_profiling(False)
        # 13B Q4_1 512-token prompt eval (best of 3): the Q4_1 MFMA matmuls (mm_mfma41.hip)
        ptoks13 = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, n_ctx)], np.int32)
        best13 = 1e30
        for _ in range(3):
            coord.barrier()
            t0 = time.perf_counter()
            m13.eval(ptoks13, 0)
            best13 = min(best13, coord.max(time.perf_counter() - t0))
        m13.close()
        E13, F13 = 5120, 13824
        fmas13 = 2.0 * 40 * (4 * E13 * E13 + 3 * E13 * F13) / 4 * len(ptoks13)   # 16 chain FMAs per 32 weights
        prompt13 = {"value": n_gpus * len(ptoks13) / best13, "unit": "tok/s", "n_tokens": len(ptoks13),
                    "ms": best13 * 1e3, "a16_image_bytes": image13,
                    "path": "matrix cores (chain partials, cross-term sums, scale products) + VALU fp32 chains "
                            "(ggml_vec_dot_q4_1); bit-identical to the AVX2 reference",
                    "roofline": {"bound": "valu-fp32 (the reference's sequential fp32 FMA chains)",
                                 "achieved": 2 * fmas13 / best13 / 1e12, "peak": VALU_FP32_TFLOPS,
                                 "unit": "TFLOP/s", "frac": 2 * fmas13 / best13 / 1e12 / VALU_FP32_TFLOPS,
                                 "fp32_chain_fmas": fmas13}}
        k13 = {k: {"avg_us": v["ms"] / v["launches"] * 1e3,
                   "gbs": v["bytes"] / v["launches"] / (v["ms"] / v["launches"] * 1e-3) / 1e9 if v["bytes"] else None}
               for k, v in p13.items() if v["launches"]}
        r13 = args.steps_13b / t13
        q41 = {"value": n_gpus * r13, "unit": "tok/s", "steps": args.steps_13b,
               "workload": "LLaMA-13B Q4_1 (synthetic, seed 2) single-stream greedy decode, %d steps at positions "
                           "spread evenly over 16..%d (window filled first), n_ctx %d" % (args.steps_13b, n_ctx - 1, n_ctx),
               "stream_check": stream13,
               "model_bytes_per_token": MODEL_BYTES_13B_Q41,
               "frac_hbm_roofline": r13 * MODEL_BYTES_13B_Q41 / 1e9 / HBM_PEAK_GBS,
               "roofline_tok_s": HBM_PEAK_GBS * 1e9 / MODEL_BYTES_13B_Q41, "kernels": k13,
               "prompt_eval": prompt13}
        if rank == 0 and ws == 1 and not args.no_cpu_baseline:
            q41["cpu_baseline"] = cpu_baseline(path13, args.cpu_budget / 2, label="13B Q4_1", prompt=False,
                                               seg_steps=8)
    # N > 1: LLaMA-65B split by layers over the ranks (RCCL send/recv of
    # the residual stream between stages)
    split = None
    if (ws > 1 or args.split_rehearse) and not args.no_split:
        split = layer_split(args, coord)
    d65 = None
    if ws == 1 and not args.no_65b:
        d65 = decode_65b(args, coord, n_ctx, ptoks)
    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.model, args.cpu_budget)

    if rank != 0:
        return None
    out = {
        "metric": "decode tok/s + prompt-eval tok/s, LLaMA-7B Q4_0; % HBM roofline",
        "value": value, "unit": "tok/s", "n_gpus": n_gpus, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": value / REF_PUBLISHED_TOKS,
        "vs_baseline_note": "vs_baseline divides by the README's published 7B Q4_0 CPU figure (16.3 tok/s, Apple "
                            "Silicon, BASELINE.md section 1); vs_cpu_baseline divides by the reference build timed "
                            "on this box's host cores in this run (cpu_baseline)",
        "vs_cpu_baseline": (value / n_gpus / cpu["value"]) if cpu else None,
        "dtype": "i4xi4->f32 (Q4_0 blocks, exact int dots, fp32 FMA chains)",
        "data": "synthetic (seeded ggjt 7B Q4_0, lvk-gen-model seed 1)",
        "config": {"workload": "LLaMA-7B Q4_0 single-stream decode: 16-token prompt then %d greedy decode "
                               "steps at positions %s, n_ctx 512, f16 KV" % (args.steps, positions),
                   "n_ctx": n_ctx,
                   "parallelism": "replicas" if n_gpus > 1 else "single-gpu"},
        "roofline": roofline,
        "step_roofline": {"model_bytes_per_token": MODEL_BYTES_7B, "achieved_gbs": step_gbs,
                          "frac": step_gbs / HBM_PEAK_GBS, "roofline_tok_s": HBM_PEAK_GBS * 1e9 / MODEL_BYTES_7B},
        "prompt_eval": prompt,
        "decode_greedy_device": greedy,
        "decode_13b_q4_1": q41,
        "decode_65b_q4_0": d65,
        "layer_split": split,
        "kernels": kernels,
        "cpu_baseline": cpu,
        "load_s": load_s,
    }
    out["checks"] = collect_checks(out)
    return out


def collect_checks(out):
    """every correctness field the legs recorded: a false one marks the line invalid (bench.py
    exits non-zero after printing it)"""
    failed = []

    def walk(node, path):
        if isinstance(node, dict):
            for k, v in node.items():
                if k in CHECK_KEYS and v is not True:
                    failed.append(path + k)
                walk(v, path + k + ".")

    walk(out, "")
    return {"passed": not failed, "failed": failed, "keys": sorted(CHECK_KEYS)}


CHECK_KEYS = {"digests_equal", "tokens_match_eval_greedy", "logits_bit_identical_every_step", "match",
              "prompt_logits_bit_identical", "tokens_equal"}


def fill_window(m, ptoks, n_ctx):
    """16-token prompt, then greedy steps over positions 16..n_ctx-1 (every K / V row of the
    window exists before a timed step reads it); returns the greedy token after the prompt"""
    import numpy as np
    tok = int(np.argmax(m.eval(ptoks, 0)[-1]))
    for p in range(len(ptoks), n_ctx):
        tok = int(np.argmax(m.eval([tok], p, copy=False)[-1]))
    return int(np.argmax(m.eval(ptoks, 0)[-1]))


def spread_pos(i, steps, n_ctx, first=16):
    """position of timed step i: K steps spread evenly over first..n_ctx-1 (K = the window: each
    once, in order; more: wrapping)"""
    win = n_ctx - first
    return first + (i * win // steps if steps <= win else i % win)


def stream_check(m, ptoks, n):
    """teacher-forced stream check: seeded non-repeating tokens through per-step llama_eval and
    through lvk_decode_chain; every step's device logits digest must equal the digest of the
    per-step logits row"""
    import lvk
    from oracle_lib import forced_tokens
    if n <= 0:
        return None
    seq_f = forced_tokens(n)
    m.eval(ptoks, 0)
    want = [lvk.logits_digest(m.eval([int(t)], len(ptoks) + i)[-1]) for i, t in enumerate(seq_f)]
    m.eval(ptoks, 0)
    _, got = m.decode_chain(seq_f, len(ptoks))
    return {"steps": len(seq_f), "positions": "%d..%d" % (len(ptoks), len(ptoks) + len(seq_f) - 1),
            "tokens": "oracle_lib.forced_tokens (seeded, non-repeating)",
            "digests_equal": got.tolist() == want, "first_digests": [hex(d) for d in want[:3]]}


if __name__ == "__main__":
    main()
