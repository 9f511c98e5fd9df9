"""The box's CPU limits and whether a command gets throttled: prints the
cgroup's cpu.max / cpuset / cpu.stat before and after running the command as
a child process (its stdout is passed through).
usage: python tools/cgroup_probe.py CMD [ARGS...]"""
import os
import subprocess
import sys


def read(p):
    try:
        with open(p) as f:
            return f.read().strip()
    except OSError as e:
        return f"({e.__class__.__name__})"


def stat():
    out = {}
    for line in read("/sys/fs/cgroup/cpu.stat").splitlines():
        parts = line.split()
        if len(parts) == 2 and parts[1].isdigit():
            out[parts[0]] = int(parts[1])
    return out


def main():
    print("cpu.max:", read("/sys/fs/cgroup/cpu.max"))
    print("cpuset.cpus.effective:", read("/sys/fs/cgroup/cpuset.cpus.effective"))
    print("sched_getaffinity:", len(os.sched_getaffinity(0)), "cpus; os.cpu_count:", os.cpu_count())
    a = stat()
    rc = subprocess.call(sys.argv[1:])
    b = stat()
    print("cpu.stat delta:", {k: b[k] - a.get(k, 0) for k in b})
    return rc


if __name__ == "__main__":
    sys.exit(main())
