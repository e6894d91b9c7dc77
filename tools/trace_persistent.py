"""Dev tool: phase timeline of the persistent decode kernel (trace build,
lib/trace/libllama_vk_amd.so built with -DLVK_DP_TRACE).  Runs a few 7B decode steps,
reads the per-workgroup phase stamps of the last one and prints where a layer's time
goes (mean over workgroups and layers 1..L-2), the edge latencies (last producer ->
first / last consumer) and the ring stall cycles."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('LVK_LIB', os.path.join(ROOT, 'llama.vk_amd', 'lib', 'trace', 'libllama_vk_amd.so'))
sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk

EV = ['start', 'x_ready', 'act', 'qkv_done', 'head_ready', 'attn_done', 'attn_all', 'wo_act', 'wo_done',
      'x1_ready', 'w13_act', 'w13_done', 'u_ready', 'w2_act', 'w2_done', 'end']


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else '/tmp/lvk_bench/llama-7b-q4_0.bin'
    pos = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        lvk.gen_model(path, vocab=os.path.join(ROOT, 'tests', 'golden', 'vocab32000.bin'),
                      n_embd=4096, n_head=32, n_layer=32, ftype=2, seed=1)
    m = lvk.Llama(path, n_ctx=512)
    hp = lvk.model_hparams(path)
    L = hp['n_layer']
    toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, 16)], np.int32)
    tok = int(np.argmax(m.eval(toks, 0)[-1]))
    for i in range(5):
        tok = int(np.argmax(m.eval([tok], pos + i)[-1]))
    m.set_profiling(True)
    m.reset_profile()
    tok = int(np.argmax(m.eval([tok], pos + 5)[-1]))
    kernel_us = m.profile()['decode']['ms'] * 1e3
    m.set_profiling(False)
    n = lvk.lib.lvk_dp_trace
    n.restype = C.c_int
    row = 96 * 16 + 16
    stamps = np.zeros(256 * row, np.uint64)
    stalls = np.zeros(256 * 16, np.uint64)
    rc = n(stamps.ctypes.data_as(C.c_void_p), stalls.ctypes.data_as(C.c_void_p))
    assert rc == row, rc
    m.close()
    st = stamps.reshape(256, row)[:, :96 * 16].reshape(256, 96, 16).astype(np.int64)
    NB = 256
    # s_memrealtime runs per XCD (no common epoch): durations within a workgroup, and
    # cross-workgroup comparisons only among b = 0 mod 8 (one XCD under round-robin dealing)
    dur = st[:, L, 15] - st[:, 0, 0]
    tick_us = kernel_us / float(np.median(dur))
    us = (st - st[:, :1, :1]) * tick_us
    out = {'kernel_us': kernel_us, 'tick_ns': tick_us * 1e3, 'layers': L, 'pos': pos}
    lay = us[:, 1:L - 1, :]
    natt = 4 * hp['n_head']

    def mean_d(a, b, wgs=slice(None)):
        return float(np.mean(lay[wgs, :, b] - lay[wgs, :, a]))
    per = {
        'x_wait': mean_d(0, 1), 'qkv_act': mean_d(1, 2), 'qkv_rows': mean_d(2, 3),
        'head_wait(att)': mean_d(3, 4, slice(0, natt)), 'attention(att)': mean_d(4, 5, slice(0, natt)),
        'wo_wait': mean_d(5, 6), 'wo_act': mean_d(6, 7), 'wo_rows+arrive': mean_d(7, 8),
        'x1_wait': mean_d(8, 9), 'w13_act': mean_d(9, 10), 'w13_rows+arrive': mean_d(10, 11),
        'u_wait': mean_d(11, 12), 'w2_act': mean_d(12, 13), 'w2_rows+arrive': mean_d(13, 14),
    }
    per['layer'] = float(np.mean(us[:, 2:L, 0] - us[:, 1:L - 1, 0]))
    out['phase_mean_us'] = {k: round(v, 2) for k, v in per.items()}
    # edges: last producer done -> first consumer saw it / last consumer saw it
    edges = {}
    for name, a, b_, prod in [('qkv->attn', 3, 4, slice(None)), ('attn->wo', 5, 6, slice(0, natt)),
                              ('wo->w13', 8, 9, slice(None)), ('w13->w2', 11, 12, slice(None)),
                              ('w2->qkv', 14, 1, slice(None))]:
        if name == 'w2->qkv':
            lastp = lay[::8, :-1, 14].max(axis=0)
            firstc = lay[::8, 1:, 1].min(axis=0)
            lastc = lay[::8, 1:, 1].max(axis=0)
        else:
            cons = slice(0, natt, 8) if name == 'qkv->attn' else slice(None, None, 8)
            prod = slice(prod.start, prod.stop, 8)
            lastp = lay[prod, :, a].max(axis=0)
            firstc = lay[cons, :, b_].min(axis=0)
            lastc = lay[cons, :, b_].max(axis=0)
        edges[name] = {'first': round(float(np.mean(firstc - lastp)), 2), 'last': round(float(np.mean(lastc - lastp)), 2)}
    out['edge_us'] = edges
    # per-phase spread: first and last workgroup to finish a phase
    spread = {}
    for name, k in [('qkv_done', 3), ('attn_done', 5), ('wo_done', 8), ('w13_done', 11), ('w2_done', 14)]:
        wgs = slice(0, natt, 8) if k == 5 else slice(None, None, 8)
        spread[name] = round(float(np.mean(lay[wgs, :, k].max(axis=0) - lay[wgs, :, k].min(axis=0))), 2)
    out['finish_spread_us'] = spread
    # s_memtime counts shader clocks: reported as a fraction of the token (at 2.4 GHz)
    sl = stalls.reshape(256, 16).astype(np.float64) / 2400.0
    out['stall_us_mean_per_wave'] = {'consumer_full_wait': round(float(sl[:, :8].mean()), 1),
                                     'loader_free_wait': round(float(sl[:, 8:10].mean()), 1)}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
