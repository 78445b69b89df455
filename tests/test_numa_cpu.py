"""NUMA placement of the host-staged path (src/io/numa.cpp): the GPU's node is
resolved from sysfs (bus/pci/devices/<bus id>/numa_node, then the node's
cpulist) — checked against a fake sysfs tree, no GPU needed."""
import pytest

from cuda_mapreduce_amd import ops


def _tree(root, bus, node, cpulist):
    d = root / "bus" / "pci" / "devices" / bus
    d.mkdir(parents=True)
    (d / "numa_node").write_text(f"{node}\n")
    if node >= 0:
        n = root / "devices" / "system" / "node" / f"node{node}"
        n.mkdir(parents=True)
        (n / "cpulist").write_text(cpulist + "\n")


@pytest.mark.parametrize("cpulist,want", [
    ("0-3", [0, 1, 2, 3]),
    ("8-15,24-31", list(range(8, 16)) + list(range(24, 32))),
    ("5", [5]),
    ("0-1,4,6-7", [0, 1, 4, 6, 7]),
])
def test_numa_of_pci(tmp_path, cpulist, want):
    _tree(tmp_path, "0000:c5:00.0", 1, cpulist)
    node, cpus = ops.numa_of_pci("0000:C5:00.0", str(tmp_path))  # HIP may report upper-case hex
    assert node == 1 and cpus == want


def test_numa_unknown(tmp_path):
    _tree(tmp_path, "0000:05:00.0", -1, "")
    assert ops.numa_of_pci("0000:05:00.0", str(tmp_path)) == (-1, [])
    assert ops.numa_of_pci("0000:99:00.0", str(tmp_path)) == (-1, [])  # no such device
