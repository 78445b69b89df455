"""Per-step cost of the cross-GPU merge protocol measured at ONE rank (RCCL world
size 1 with WC_MERGE_ALWAYS=1): finalize with and without the merge on the bench's
1 GiB Zipf text.  An upper-bound proxy for the fixed (latency) part of the merge
on a real multi-GPU node; the xGMI transfer itself is not included."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cuda_mapreduce_amd import ops  # noqa: E402

vocab = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
uid = ops.Comm.unique_id()
comm = ops.Comm(uid, 0, 1, 0)
for mode in (0, 1):
    e = ops.Engine(device=0, merge_mode=mode)
    e.synth_device(1 << 30, seed=1, vocab=vocab)
    res = {}
    for label, c in (("local", None), ("merge", comm)):
        ts = []
        for i in range(6):
            e.reset()
            e.count_resident(1 << 30)
            t0 = time.perf_counter()
            e.finalize_device(c)
            ts.append((time.perf_counter() - t0) * 1e3)
        res[label] = min(ts[1:])
    print(f"merge_mode={mode} vocab={vocab}: finalize local {res['local']:.3f} ms, with merge protocol "
          f"{res['merge']:.3f} ms (+{res['merge'] - res['local']:.3f} ms)", flush=True)
    e.close()
comm.close()
