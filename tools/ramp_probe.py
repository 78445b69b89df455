"""Per-job time of the first 200 jobs on a fresh engine (1 GiB resident
synthetic text): does the short driver run (5 warm-up + 20 timed jobs) see a
ramp?  python tools/ramp_probe.py"""
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from cuda_mapreduce_amd.ops import Engine  # noqa: E402

n = 1 << 30
with Engine(device=0) as e:
    e.synth_device(n, first_segment=0, seed=1, vocab=100000)
    e.sync()
    ts = []
    for j in range(200):
        t0 = time.perf_counter()
        e.job_resident(n)
        ts.append(time.perf_counter() - t0)
        if j < 40 and j % 3 == 0:  # device time per stage of this job (stage events are on)
            st = e.stats()
            d = st["device_ms"]
            print("job %3d: wall %.4f ms, device %.4f (map %.4f reduce %.4f finalize %.4f idle %.4f) order %d" % (
                j, ts[-1] * 1e3, d["total"], d["map"], d["reduce"], d["finalize"], d["idle"], st["order_path"]),
                flush=True)
    for a in range(0, 200, 10):
        w = ts[a:a + 10]
        print("jobs %3d-%3d: %.4f ms/job (min %.4f)" % (a, a + 9, sum(w) / len(w) * 1e3, min(w) * 1e3), flush=True)
