"""Rank -> GPU -> NUMA node -> CPU binding (parallel/affinity.py) against a fake sysfs."""
import os

from tensorhive_fixed_amd.parallel import affinity as A


def _sysfs(tmp_path, gpus):
    """gpus: list of (kfd node id, bus, numa node); two NUMA nodes with 8 CPUs each."""
    kfd, pci, nodes = tmp_path / "kfd", tmp_path / "pci", tmp_path / "node"
    (kfd / "0").mkdir(parents=True)
    (kfd / "0" / "properties").write_text("simd_count 0\nlocation_id 0\n")  # the CPU node
    for nid, bus, numa in gpus:
        d = kfd / str(nid)
        d.mkdir()
        d.joinpath("properties").write_text(f"cpu_cores_count 0\nsimd_count 1024\nlocation_id {bus << 8}\ndomain 0\n")
        b = pci / f"0000:{bus:02x}:00.0"
        b.mkdir(parents=True)
        (b / "numa_node").write_text(f"{numa}\n")
    for n, cpus in ((0, "0-7"), (1, "8-15")):
        (nodes / f"node{n}").mkdir(parents=True)
        (nodes / f"node{n}" / "cpulist").write_text(cpus + "\n")
    return kfd, pci, nodes


def test_cpulist_round_trip():
    assert A.parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert A.format_cpulist([11, 10, 8, 3, 2, 1, 0]) == "0-3,8,10-11"


def test_kfd_order_and_visible_devices(tmp_path):
    # KFD node order is HIP's order, whatever the bus numbers are
    kfd, pci, nodes = _sysfs(tmp_path, [(2, 0x75, 0), (3, 0x05, 0), (4, 0xf5, 1), (5, 0x85, 1)])
    none = tmp_path / "no-dri"
    assert A.kfd_gpu_bdfs(kfd, none) == ["0000:75:00.0", "0000:05:00.0", "0000:f5:00.0", "0000:85:00.0"]
    # a container that can open only two of the render nodes: HIP enumerates those two
    for nid, minor in ((2, 128), (3, 129), (4, 130), (5, 131)):
        props = kfd / str(nid) / "properties"
        props.write_text(props.read_text() + f"drm_render_minor {minor}\n")
    dri = tmp_path / "dri"
    dri.mkdir()
    for minor in (129, 131):
        (dri / f"renderD{minor}").write_text("")
    assert A.kfd_gpu_bdfs(kfd, dri) == ["0000:05:00.0", "0000:85:00.0"]
    assert A.visible_physical(4, {}) == [0, 1, 2, 3]
    assert A.visible_physical(4, {"HIP_VISIBLE_DEVICES": "3,2"}) == [3, 2]
    assert A.visible_physical(4, {"ROCR_VISIBLE_DEVICES": "1,2,3", "HIP_VISIBLE_DEVICES": "2"}) == [3]
    p = A.plan(1, 2, "numa", {"HIP_VISIBLE_DEVICES": "1,0"}, kfd, pci, nodes, dri)
    assert p["bdf"] == "0000:05:00.0" and p["numa_node"] == 0 and p["cpus"] == "0-7"


def test_exclusive_mode_splits_a_nodes_cpus(tmp_path):
    kfd, pci, nodes = _sysfs(tmp_path, [(2, 0x05, 0), (3, 0x15, 0), (4, 0x25, 1), (5, 0x35, 1)])
    got = [A.plan(r, 4, "exclusive", {}, kfd, pci, nodes, tmp_path / "no-dri")["cpus"] for r in range(4)]
    assert got == ["0-3", "4-7", "8-11", "12-15"]


def test_no_topology_is_a_no_op(tmp_path):
    p = A.plan(0, 1, "numa", {}, tmp_path / "none", tmp_path, tmp_path)
    assert p["applied"] is False and p["bdf"] is None and p["reason"]


def test_bind_applies_the_mask(tmp_path, monkeypatch):
    kfd, pci, nodes = _sysfs(tmp_path, [(2, 0x05, 0)])
    allowed = sorted(os.sched_getaffinity(0))
    (nodes / "node0" / "cpulist").write_text(A.format_cpulist(allowed[:1]) + "\n")
    monkeypatch.setattr(A, "KFD_NODES", kfd)
    monkeypatch.setattr(A, "PCI", pci)
    monkeypatch.setattr(A, "NODES", nodes)
    monkeypatch.setattr(A, "DRI", tmp_path / "no-dri")
    calls = []
    monkeypatch.setattr(os, "sched_setaffinity", lambda pid, cpus: calls.append(set(cpus)))
    p = A.bind(0, 1, "numa")
    assert p["applied"] and calls == [{allowed[0]}] and p["cpus"] == str(allowed[0])
    assert A.bind(0, 1, "none") == {"mode": "none", "applied": False}
