"""tools/merge_rank_cost.py on synthetic kernel traces (CPU): per-rank merge
time = the merge kernels after a rank's reduce, split by host thread, median
of the timed jobs; the two 8-GPU predictions add the wire model (largest
per-peer bytes / one xGMI link + a launch per collective) to the contended
time of the slowest rank and to the W = 1 (uncontended) time."""
import csv
import importlib.util
import json
import os

TOOL = os.path.join(os.path.dirname(__file__), "..", "tools", "merge_rank_cost.py")


def load_tool():
    spec = importlib.util.spec_from_file_location("merge_rank_cost", TOOL)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def write_run(d, tag, W, merge_us_by_rank, peer_bytes, collectives, jobs=5):
    """A bench JSON + a kernel trace: every rank runs `jobs` jobs of
    hot_sample -> map -> reduce -> merge kernels (two per job, splitting the time)."""
    os.makedirs(os.path.join(d, tag, "host"), exist_ok=True)
    info = {"virtual_ranks": W, "config": {"vocab": 100000, "merge": "shuffle"}, "validated": True,
            "merges_planned_rank0": jobs, "merge_redos_rank0": 0,
            "merge_wire": [{"merge_collectives": collectives, "merge_sent_bytes": 3 * peer_bytes,
                            "merge_peer_bytes": peer_bytes, "merge_root_recv_bytes": 0} for _ in range(W)]}
    with open(os.path.join(d, tag + ".json"), "w") as f:
        f.write(json.dumps(info) + "\n")
    rows = []
    for rank, us in enumerate(merge_us_by_rank):
        t = 1000 * rank
        for _ in range(jobs):
            for name, dur in (("wc::dev::wc_hot_sample(x)", 10.0), ("void wc::dev::wc_map<false>(x)", 500.0),
                              ("wc::dev::wc_reduce_buckets(x)", 200.0), ("wc::dev::wc_owner_scatter(x)", us / 2),
                              ("wc::dev::wc_mrow_insert(x)", us / 2), ("wc::dev::wc_fo_sort(x)", 7.0)):
                rows.append({"Thread_Id": str(100 + rank), "Kernel_Name": name, "Start_Timestamp": str(int(t * 1e3)),
                             "End_Timestamp": str(int((t + dur) * 1e3))})
                t += dur + 1.0
    with open(os.path.join(d, tag, "host", "run_kernel_trace.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)


def test_merge_rank_cost_table(tmp_path, capsys):
    m = load_tool()
    write_run(str(tmp_path), "w1_v100000_shuffle", 1, [60.0], 0, 3)
    write_run(str(tmp_path), "w2_v100000_shuffle", 2, [300.0, 200.0], 1_530_000, 3)
    m.main(str(tmp_path))
    out = capsys.readouterr().out.strip().splitlines()
    rows = {int(r.split("|")[1]): [c.strip() for c in r.split("|")[1:-1]] for r in out[2:]}
    assert set(rows) == {1, 2}
    w2 = rows[2]
    assert float(w2[3]) == 300.0 and float(w2[4]) == 250.0  # slowest rank, mean rank (fo_sort not counted)
    wire = 1_530_000 / (m.LINK_GBS * 1e3) + m.COLL_US * 3  # 10 us + 3 collective launches
    assert abs(float(w2[8]) - (300.0 + wire)) < 0.1  # contended kernels + wire
    assert abs(float(w2[9]) - (60.0 + wire)) < 0.1  # W = 1 kernels + wire
    assert abs(float(rows[1][9]) - (60.0 + m.COLL_US * 3)) < 0.1
