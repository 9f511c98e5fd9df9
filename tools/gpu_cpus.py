"""Print a CPU list of N physical cores (one hardware thread each) on the NUMA
node of GPU 0 -- for taskset A/B runs of host-thread placement.
usage: python tools/gpu_cpus.py [N]"""
import glob
import os
import sys

import torch


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    p = torch.cuda.get_device_properties(0)
    bus = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    node = int(open(f"/sys/bus/pci/devices/{bus}/numa_node").read())
    picked, seen = [], set()
    for cpu in sorted(int(d.rsplit("cpu", 1)[1]) for d in glob.glob(f"/sys/devices/system/node/node{node}/cpu[0-9]*")):
        core = open(f"/sys/devices/system/cpu/cpu{cpu}/topology/core_id").read().strip()
        pkg = open(f"/sys/devices/system/cpu/cpu{cpu}/topology/physical_package_id").read().strip()
        if (pkg, core) in seen or cpu not in os.sched_getaffinity(0):
            continue
        seen.add((pkg, core))
        picked.append(cpu)
        if len(picked) == n:
            break
    print(",".join(map(str, picked)))


if __name__ == "__main__":
    main()
