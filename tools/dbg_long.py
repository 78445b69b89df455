import collections, os, sys
sys.path.insert(0, os.getcwd())
from cuda_mapreduce_amd import ops
n = 128 << 20
chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 32 << 20
with ops.Engine(device=0, chunk_bytes=chunk) as e:
    e.synth_device(n, first_segment=0, seed=3, vocab=1_000_000, zipf_s=1.0, long_frac=0.3)
    e.count_resident(n)
    got = e.result()
    st = e.stats()
want = ops.cpu_count_synth(n, 0, 3, 1_000_000, 1.0, 0, 16, 0.3)
g = collections.Counter(got.words)
dups = [w for w, c in g.items() if c > 1]
gw = dict(zip(got.words, got.counts)); ww = dict(zip(want.words, want.counts))
extra = [w for w in gw if w not in ww]
missing = [w for w in ww if w not in gw]
bad = [w for w in ww if w in gw and gw[w] != ww[w]]
print("env RED_Q", os.environ.get("WC_RED_Q"), "chunk", chunk, "stats", {k: st[k] for k in ("log2_buckets", "table_splits", "map_reruns", "chunks") if k in st})
print("got", len(got.words), "want", len(want.words), "dups", len(dups), "extra", len(extra), "missing", len(missing), "badcount", len(bad))
for w in dups[:3]: print(" dup", w, len(w), [gc for gw_, gc in zip(got.words, got.counts) if gw_ == w], ww.get(w))
for w in bad[:3]: print(" bad", w, len(w), gw[w], ww[w])
print(" dup lens", collections.Counter(len(w) >= 16 for w in dups))
