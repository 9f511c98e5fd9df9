"""Host-stage CPU profile of the bench step (C3) with tools/libsampler.so.

usage: python tools/sampler.py OUT_PREFIX [steps] [contig_bp]
Runs the bench step (FASTA load, upload, scan, post-processing, write) under
SIGPROF sampling and prints the top functions (file offsets symbolised with nm)."""
import bisect
import collections
import ctypes
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "bwt-algorithm_amd")]


def symbols(path):
    tab = []
    for extra in ([], ["-D"]):
        out = subprocess.run(["nm", "-C", "--defined-only"] + extra + [path], stdout=subprocess.PIPE,
                             stderr=subprocess.DEVNULL, text=True).stdout
        for line in out.splitlines():
            parts = line.split(" ", 2)
            if len(parts) == 3 and parts[1] in "tTwWiI":
                tab.append((int(parts[0], 16), parts[2]))
        if tab:
            break
    tab.sort()
    return tab


def load_delta(path):
    """vaddr - file offset of the executable LOAD segment (nm prints vaddrs)."""
    out = subprocess.run(["readelf", "-lW", path], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                         text=True).stdout
    for line in out.splitlines():
        f = line.split()
        if f and f[0] == "LOAD" and "E" in line.split()[-2:-1][0] if len(f) > 7 else False:
            return int(f[2], 16) - int(f[1], 16)
    return 0


def inclusive(path, tabs):
    """Samples per function anywhere on the stack (each function once per sample)."""
    if not os.path.exists(path):
        return collections.Counter()
    chains = [line.split() for line in open(path)]
    addrs = {}
    for ch in chains:
        for fr in ch:
            mod, off = fr.rsplit(":", 1)
            if "libbwtmi" in mod:
                addrs.setdefault(mod, set()).add(int(off, 16))
    names = {}
    for mod, offs in addrs.items():
        delta = tabs[mod][1] if mod in tabs else load_delta(mod)
        offs = sorted(offs)
        out = subprocess.run(["addr2line", "-e", mod, "-C", "-f", "-i", "-a"],
                             input="\n".join(hex(o + delta) for o in offs), stdout=subprocess.PIPE,
                             text=True).stdout.splitlines()
        cur, k = None, 0
        while k < len(out):
            line = out[k]
            if line.startswith("0x"):
                cur = int(line, 16) - delta
                names[(mod, cur)] = []
                k += 1
                continue
            fn = line.replace("(anonymous namespace)::", "").split("(")[0].strip()
            if not fn.startswith(("std::", "__", "operator", "void std::")):
                names[(mod, cur)].append(fn[:100])
            k += 2   # function line, then file:line
    incl = collections.Counter()
    for ch in chains:
        if not any("libbwtmi" in fr for fr in ch):
            continue   # idle / other threads: only samples inside the library count
        incl["(samples in libbwtmi)"] += 1
        seen = set()
        for fr in ch:
            mod, off = fr.rsplit(":", 1)
            for fn in names.get((mod, int(off, 16)), [os.path.basename(mod)[:20]]):
                seen.add(fn)
        for fn in seen:
            incl[fn] += 1
    return incl


def report(prefix, raw):
    tabs = {}
    by_fn = collections.Counter()
    for line in open(raw):
        mod, off, cnt = line.split()
        off, cnt = int(off, 16), int(cnt)
        name = os.path.basename(mod)
        if os.path.exists(mod) and (".so" in mod or "libbwtmi" in mod):
            if mod not in tabs:
                tabs[mod] = (symbols(mod), load_delta(mod))
            tab, delta = tabs[mod]
            k = bisect.bisect_right(tab, (off + delta, "\xff")) - 1
            name = tab[k][1] if k >= 0 else name
        by_fn[f"{os.path.basename(mod)[:18]}: {name}"] += cnt
    tot = sum(by_fn.values())
    # source lines of the hottest libbwtmi addresses (needs -g; addr2line -i shows the inline chain)
    hot = collections.Counter()
    for line in open(raw):
        mod, off, cnt = line.split()
        if "libbwtmi" in mod:
            hot[(mod, int(off, 16))] += int(cnt)
    lines = collections.Counter()
    top = hot.most_common(400)
    if top:
        mod = top[0][0][0]
        delta = tabs[mod][1] if mod in tabs else 0
        for ((m, off), c) in top:   # innermost inlined frame of each address
            r = subprocess.run(["addr2line", "-e", m, "-C", "-f", hex(off + delta)], stdout=subprocess.PIPE,
                               text=True).stdout.splitlines()
            if len(r) >= 2:
                lines[f"{r[1].split('/')[-1]} {r[0][:60]}"] += c
    incl = inclusive(raw + ".chains", tabs)
    with open(prefix + ".txt", "w") as f:
        for name, c in by_fn.most_common(80):
            f.write(f"{100.0 * c / tot:6.2f}% {c:8d} {name[:160]}\n")
        f.write("\n-- hottest source lines (libbwtmi)\n")
        for name, c in lines.most_common(60):
            f.write(f"{100.0 * c / tot:6.2f}% {c:8d} {name}\n")
        f.write("\n-- inclusive (frame-pointer chains; inlined frames from addr2line -i)\n")
        for name, c in incl.most_common(80):
            f.write(f"{100.0 * c / tot:6.2f}% {c:8d} {name[:150]}\n")
    print(open(prefix + ".txt").read()[:6000])


def main():
    prefix = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 100_000_000
    lib = ctypes.CDLL(os.path.join(REPO, "tools", "libsampler.so"))
    from bwtmi import _lib, synth
    from bwtmi.records import Job
    ctx = _lib.ctx(0)
    fa = os.path.join(tempfile.gettempdir(), "sampler_c3.fa")
    synth.write_fasta(fa, [n], 0.0)
    out = os.path.join(tempfile.gettempdir(), "sampler_c3.tab")
    job = Job(min_copies=3, max_unit_len=120, show_progress=True, tier2=True, build_index=True, sa_sample=32)

    def step():
        job.reset()
        job.load_fasta(fa, 30)
        job.upload(ctx)
        job.scan(ctx)
        job.postprocess()
        job.write("strfinder", out)
        job.wait(ctx)

    step()
    print("threads sampled:", lib.sampler_start(2000), flush=True)
    t0 = time.time()
    for _ in range(steps):
        step()
    dt = time.time() - t0
    raw = prefix + ".raw"
    ns = lib.sampler_stop(raw.encode())
    print(f"{steps} steps {dt * 1e3 / steps:.1f} ms/step, {ns} samples", flush=True)
    report(prefix, raw)
    os.unlink(fa)
    os.unlink(out)


if __name__ == "__main__":
    main()
