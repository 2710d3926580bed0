"""NUMA pinning of a rank (parallel/affinity.py) on a synthetic sysfs tree."""
import os

from semantic_segmentation_server_amd.parallel import affinity as A


def _tree(root, gpus):
    # KFD topology: node 0 = CPU, nodes 1.. = GPUs with PCI location / domain
    os.makedirs(f"{root}/class/kfd/kfd/topology/nodes/0")
    open(f"{root}/class/kfd/kfd/topology/nodes/0/properties", "w").write("simd_count 0\ncpu_cores_count 8\n")
    for i, (bus, numa) in enumerate(gpus, 1):
        d = f"{root}/class/kfd/kfd/topology/nodes/{i}"
        os.makedirs(d)
        open(f"{d}/properties", "w").write(f"simd_count 1024\nlocation_id {bus << 8}\ndomain 0\n")
        p = f"{root}/bus/pci/devices/0000:{bus:02x}:00.0"
        os.makedirs(p)
        open(f"{p}/numa_node", "w").write(f"{numa}\n")
    cpus = sorted(os.sched_getaffinity(0))
    half = max(1, len(cpus) // 2)
    for n, sel in ((0, cpus[:half]), (1, cpus[half:] or cpus[:1])):
        os.makedirs(f"{root}/devices/system/node/node{n}")
        open(f"{root}/devices/system/node/node{n}/cpulist", "w").write(",".join(map(str, sel)))
    return cpus, half


def test_cpulist_parse():
    assert A.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}


def test_pin_to_gpu_numa(tmp_path, monkeypatch):
    root = str(tmp_path)
    cpus, half = _tree(root, [(0x11, 0), (0x91, 1)])
    assert A.gpu_pci_addresses(root) == ["0000:11:00.0", "0000:91:00.0"]
    assert A.gpu_numa_node(1, root) == 1
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "1,0")
    assert A.gpu_numa_node(0, root) == 1            # local rank 0 -> device 1
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES")
    before = os.sched_getaffinity(0)
    try:
        got = A.pin_to_gpu_numa(0, root)
        if len(cpus) > 1:
            assert got == set(cpus[:half]) and os.sched_getaffinity(0) == set(cpus[:half])
    finally:
        os.sched_setaffinity(0, before)
    assert A.pin_to_gpu_numa(0, str(tmp_path / "missing")) is None
