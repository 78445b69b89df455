import sys, numpy as np, json
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from cuda_mapreduce_amd import ops
from cuda_mapreduce_amd.ops import cpu_count
from test_gpu_engine import random_text
rng = np.random.default_rng(0)
n = int(rng.choice([1, 17, 1000, 16383, 16384, 16385, 70000, 300000, 2_000_000]))
text = random_text(rng, n, long_words=3)
print("n", n)
e = ops.Engine(device=0, chunk_bytes=1 << 22)
e.reset(); e.count_bytes(text); g = e.result()
print("stats", {k: v for k, v in e.stats().items() if not isinstance(v, (list, dict))})
w = cpu_count(text)
gd = {k: (int(c), int(f)) for k, c, f in zip(g.words, g.counts, g.first_off)}
wd = {k: (int(c), int(f)) for k, c, f in zip(w.words, w.counts, w.first_off)}
miss = [k for k in wd if k not in gd]
bad = [k for k in wd if k in gd and gd[k] != wd[k]]
print("keys got", len(gd), "want", len(wd), "missing", len(miss), "wrong", len(bad))
for k in miss[:10]: print("missing", k, wd[k], len(k))
for k in bad[:10]: print("wrong", k, gd[k], wd[k])
extra = [k for k in gd if k not in wd]
for k in extra[:10]: print("extra", k, gd[k])
