"""Cost of the cross-GPU merge protocols (shuffle = merge_mode 0, dense = 1).

Measured at ONE rank over RCCL (world size 1, the protocol forced on): finalize
of the bench's 1 GiB Zipf text without and with the merge, per protocol — the
merge's kernels, host syncs and RCCL launch latencies, but no xGMI transfer.
Then an analytic W-rank model adds the wire time of every exchange for the
same per-rank table on an MI355X node (7 xGMI links x ~153 GB/s per GPU,
point to point): all-to-all traffic to each peer rides its own link; ring
reduce-scatter / all-gather are bound by one link per step.

usage: python tools/merge_cost.py [vocab ...]   (markdown table on stdout)
"""
import os
import sys
import time

os.environ["WC_MERGE_ALWAYS"] = "1"  # run the protocol at world size 1
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cuda_mapreduce_amd import ops  # noqa: E402

LINK_GBS = 153.0   # one xGMI link, GB/s per direction
ROW_B = 40         # MRow on the wire
W_MODEL = 8


PROTOCOLS = ((0, "shuffle", None), (0, "shuffle, owner path", "0"), (1, "dense", None))


def measure(vocab, comm):
    out = {}
    for mode, name, root_rows in PROTOCOLS:
        if root_rows is None:
            os.environ.pop("WC_MERGE_ROOT_ROWS", None)
        else:
            os.environ["WC_MERGE_ROOT_ROWS"] = root_rows  # read per merge
        e = ops.Engine(device=0, merge_mode=mode)
        e.synth_device(1 << 30, seed=1, vocab=vocab)
        res = {}
        for label, c in (("local", None), ("merge", comm)):
            ts = []
            for _ in range(6):
                e.reset()
                e.count_resident(1 << 30)
                t0 = time.perf_counter()
                keys = e.finalize_device(c)
                ts.append((time.perf_counter() - t0) * 1e3)
            res[label] = min(ts[1:])
            res["keys"] = keys
        out[name] = res
        e.close()
    return out


def wire_us(V, W, dense, root):
    """Per-rank xGMI time (us) of the merge exchanges for V keys per rank, all
    ranks holding the same vocabulary (the Zipf bench: union ~= V)."""
    link = LINK_GBS * 1e3  # bytes per us
    if root:                                 # every rank sends its V rows to rank 0 on its own link
        return V * ROW_B / link
    t = V / W * ROW_B / link                 # owner exchange: V/W rows to each peer, own link each
    t += V / W * ROW_B / link                # gather of the merged dictionary to rank 0: V/W rows per owner link
    if dense:
        t += V / W * 4 / link                # ids back to the senders
        vec = V * 8 * (W - 1) / W            # ring RS and AG of one u64 vector, one link per step
        t += 4 * vec / link                  # RS(sum), RS(min), AG(cnt), AG(first)
    return t


def main():
    vocabs = [int(v) for v in sys.argv[1:]] or [100000, 1000000]
    comm = ops.Comm(ops.Comm.unique_id(), 0, 1, 0)
    print("| vocab | keys/rank | protocol | finalize local ms | finalize + merge (W=1 RCCL) ms | merge ms |"
          f" modelled xGMI wire us (W={W_MODEL}) | modelled merge ms (W={W_MODEL}) |")
    print("|---|---|---|---|---|---|---|---|")
    for vocab in vocabs:
        r = measure(vocab, comm)
        for mode, name, _ in PROTOCOLS:
            m = r[name]
            V = m["keys"]
            merge = m["merge"] - m["local"]
            root = name == "shuffle" and W_MODEL * V <= (1 << 18)  # MERGE_ROOT_MAX_ROWS
            w = wire_us(V, W_MODEL, mode == 1, root)
            print(f"| {vocab} | {V} | {name} | {m['local']:.3f} | {m['merge']:.3f} | {merge:.3f} | {w:.1f} |"
                  f" {merge + w / 1e3:.3f} |", flush=True)
    comm.close()


if __name__ == "__main__":
    main()
