"""Per-rank merge cost from kernel traces of bench.py --virtual-ranks W
(tools/merge_rank_cost.sh).  Each virtual rank is one host thread of the
process, so rocprofv3's Thread_Id splits the trace by rank.  Per rank and
timed step: the device time of the merge protocol's kernels (owner scatter,
owner-table insert / compact, id return, dense scatter, check, regions ->
columns and the merge's zeroing), NOT counting the loopback transfer kernels
(on an 8-GPU node RCCL moves those bytes over xGMI: modelled below from the
ranks' reported wire bytes) nor waits on peers.  Prediction for one MI355X
per rank: device time + sum over collectives of the largest per-peer amount /
one xGMI link (~153 GB/s, each peer pair on its own link) + ~10 us launch
latency per collective.

The W virtual ranks share ONE GPU: their merge kernels run beside the other
ranks' map / reduce kernels, so their traced durations include waiting for CUs
(the max rank's merge reads 2-8x the W = 1 cost).  The second prediction
takes the uncontended device time from the W = 1 run of the same vocabulary
and protocol (the protocol forced on: WC_MERGE_ALWAYS=1): with a shared Zipf
vocabulary each owner receives about one rank's key count whatever W, so an
owner's kernels do the W = 1 work; the wire term is the W-rank one.

usage: python tools/merge_rank_cost.py DIR   (markdown table on stdout)
"""
import csv
import glob
import json
import os
import statistics
import sys

LINK_GBS = 153.0
COLL_US = 10.0
MERGE_KERNELS = ("wc_owner_scatter", "wc_mrow_insert", "wc_mrow_compact", "wc_row_ids", "wc_scatter_ids",
                 "wc_merge_check", "wc_mrow_regions_to_cols", "wc_mrow_to_cols", "wc_owner_count")


def rank_times(trace):
    """{thread: [per-step merge kernel us]}: a job starts at the thread's
    wc_hot_sample; its merge kernels are those after its wc_reduce_* launch."""
    by_thread = {}
    for r in csv.DictReader(open(trace)):
        by_thread.setdefault(r["Thread_Id"], []).append(r)
    out = {}
    for th, rows in by_thread.items():
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        if not any("wc_map" in r["Kernel_Name"] for r in rows):
            continue  # not an engine thread
        steps, cur, after_reduce = [], None, False
        for r in rows:
            n = r["Kernel_Name"]
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            if "wc_hot_sample" in n:
                if cur is not None:
                    steps.append(cur)
                cur, after_reduce = 0.0, False
            elif "wc_reduce" in n:
                after_reduce = True
            elif after_reduce and cur is not None and (
                    any(k in n for k in MERGE_KERNELS) or "wc_zero_regions" in n):
                cur += dur
        if cur is not None:
            steps.append(cur)
        out[th] = steps
    return out


def main(d):
    rows = []
    for js in sorted(glob.glob(os.path.join(d, "*.json"))):
        tag = os.path.basename(js)[:-5]
        info = json.loads(open(js).read().strip().splitlines()[-1])
        traces = glob.glob(os.path.join(d, tag, "**", "run_kernel_trace.csv"), recursive=True)
        if not traces:
            continue
        rt = rank_times(traces[0])
        per_rank = [statistics.median(v[-4:]) for v in rt.values() if v]  # the timed (planned) steps
        wire = info.get("merge_wire", [])
        peer = max((w["merge_peer_bytes"] for w in wire), default=0)
        coll = max((w["merge_collectives"] for w in wire), default=0)
        sent = max((w["merge_sent_bytes"] for w in wire), default=0)
        dev = max(per_rank) if per_rank else float("nan")
        pred = dev + peer / (LINK_GBS * 1e3) + COLL_US * coll
        rows.append([info.get("virtual_ranks", 1), info["config"]["vocab"], info["config"]["merge"], dev,
                     statistics.mean(per_rank) if per_rank else float("nan"), coll, sent, peer, pred, float("nan"),
                     info["validated"], info.get("merges_planned_rank0", 0), info.get("merge_redos_rank0", 0)])
    solo = {(r[1], r[2]): r[3] for r in rows if r[0] == 1}
    for r in rows:
        if (r[1], r[2]) in solo:
            r[9] = solo[(r[1], r[2])] + r[7] / (LINK_GBS * 1e3) + COLL_US * r[5]
    rows.sort(key=lambda r: (r[1], r[2], r[0]))
    print("| W | keys/rank | protocol | merge kernels us (max rank, contended) | (mean rank) | collectives |"
          " bytes sent / rank | largest per-peer bytes (sum) | predicted: contended kernels + wire, us |"
          " predicted: W=1 kernels + wire, us | validated | planned / redos |")
    print("|---:|---:|---|---:|---:|---:|---:|---:|---:|---:|---|---|")
    for r in rows:
        print("| %d | %d | %s | %.1f | %.1f | %d | %d | %d | %.1f | %.1f | %s | %d / %d |" % tuple(r))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/mrc")
