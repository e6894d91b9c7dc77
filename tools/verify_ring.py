"""Dev tool (verify build): decode a deep tiny model on the persistent kernel and print
the ring chunks whose LDS bytes differ from the weight image."""
import ctypes as C
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('LVK_LIB', os.path.join(ROOT, 'llama.vk_amd', 'lib', 'verify', 'libllama_vk_amd.so'))
sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import numpy as np
import lvk
from oracle_lib import gen_model, prompt_tokens
L = int(sys.argv[1]) if len(sys.argv) > 1 else 12
os.makedirs('/tmp/lvk_chk', exist_ok=True)
path = gen_model('/tmp/lvk_chk/tiny%d.bin' % L, n_embd=256, n_head=2, n_layer=L, ftype=2, seed=1)
m = lvk.Llama(path, n_ctx=512)
m.set_decode_persistent(True)
toks = prompt_tokens(48)
tok = int(np.argmax(m.eval(toks, 0)[-1]))
try:
    m.eval([tok], 48)
    print('eval ok')
except RuntimeError as e:
    print('eval failed:', e)
buf = np.zeros(16 + 64 * 16 + 32 * 8, np.uint32)
lvk.lib.lvk_dp_verify(buf.ctypes.data_as(C.c_void_p))
print('mismatches:', buf[0])
names = ['b', 'l', 'epi', 'c', 'gi', 'slot', 'gen', 'qq', 'S', 'wave', 'grp', 'nsubc', 'FULL', 'FREE', 'mask', 'ring']
for k in range(min(int(buf[0]), 40)):
    e = buf[16 + k * 16: 32 + k * 16]
    print(' '.join('%s=%d' % (n, v) for n, v in zip(names, e)))

print('loader FREE violations:', buf[1])
for k in range(min(int(buf[1]), 32)):
    e = buf[16 + 64 * 16 + k * 8: 16 + 64 * 16 + k * 8 + 8]
    print(' '.join('%s=%d' % (n, v) for n, v in zip(['b', 'lw', 'q', 'slot', 'gen', 'FREE', 'S', 'tag'], e)))
