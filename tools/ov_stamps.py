"""Dev tool (round 6): in-kernel realtime stamps of the decode attention and the overlapped Wo
(the `make ovstamp` build, LVK_LIB=lib/ovstamp/...) for one decode step: does the Wo start while
the attention runs, and how long after the attention's last workgroup does it see the tags and
finish.  usage: LVK_OVERLAP=1|2 ov_stamps.py [n_past]"""
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("LVK_LIB", os.path.join(ROOT, "llama.vk_amd", "lib", "ovstamp", "libllama_vk_amd.so"))
sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk


def main():
    n_past = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    path = '/tmp/lvk_bench/llama-7b-q4_0.bin'
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        lvk.gen_model(path, n_embd=4096, n_head=32, n_layer=32, ftype=2, seed=1,
                      vocab=os.path.join(ROOT, 'tests', 'golden', 'vocab32000.bin'))
    m = lvk.Llama(path, n_ctx=512)
    toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, 16)], np.int32)
    tok = int(np.argmax(m.eval(toks, 0)[-1]))
    for p in range(16, n_past + 1):
        tok = int(np.argmax(m.eval([tok], p, copy=False)[-1]))
    lib = lvk.lib
    lib.lvk_probe_ovs_attn.restype = C.c_void_p
    lib.lvk_probe_ovs_wo.restype = C.c_void_p
    hip = C.CDLL("libamdhip64.so")
    att = np.zeros(128 * 1024 * 2, np.uint64)
    wo = np.zeros(128 * 1024 * 3, np.uint64)
    hip.hipMemcpy(att.ctypes.data_as(C.c_void_p), C.c_void_p(lib.lvk_probe_ovs_attn()), C.c_size_t(att.nbytes), 2)
    hip.hipMemcpy(wo.ctypes.data_as(C.c_void_p), C.c_void_p(lib.lvk_probe_ovs_wo()), C.c_size_t(wo.nbytes), 2)
    att = att.reshape(128, 1024, 2)[:32, :128].astype(np.int64)
    wo = wo.reshape(128, 1024, 3)[:32, :256].astype(np.int64)
    rows = []
    for l in range(32):
        a0, a1 = att[l, :, 0].min(), att[l, :, 1].max()
        w = wo[l]
        if not w.any():
            continue
        rows.append({"att_span": (a1 - a0) / 100, "wo_start_min_rel_att_start": (w[:, 0].min() - a0) / 100,
                     "wo_start_med_rel_att_end": (np.median(w[:, 0]) - a1) / 100,
                     "wo_wait_med_rel_att_end": (np.median(w[:, 1]) - a1) / 100,
                     "wo_wait_max_rel_att_end": (w[:, 1].max() - a1) / 100,
                     "wo_end_max_rel_att_end": (w[:, 2].max() - a1) / 100})
    out = {"overlap": os.environ.get("LVK_OVERLAP"), "n_past": n_past, "layers": len(rows)}
    for k in (rows[0].keys() if rows else []):
        out[k] = round(statistics.median(r[k] for r in rows), 2)
    print(json.dumps(out), flush=True)
    m.close()


if __name__ == '__main__':
    main()
