import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llama.vk_amd"))
import numpy as np
import lvk
graph = sys.argv[1] == "1"
m = lvk.Llama("/tmp/lvk_bench/llama-7b-q4_0.bin", n_ctx=512)
m.set_graph(graph)
lg = m.eval(np.arange(1, 17, dtype=np.int32), 0)
tok = int(np.argmax(lg[-1]))
for i in range(int(sys.argv[2]) if len(sys.argv) > 2 else 20):
    lg = m.eval([tok], 16 + i)
    tok = int(np.argmax(lg[-1]))
    print("step", i, tok, flush=True)
m.close()
print("done graph", graph)
