#!/usr/bin/env python3
"""Where the GPU sits relative to this process's CPUs, and the pinned-copy rates with the process bound to
the GPU's local CPUs (--bind local) or not.  PCIe DMA to pinned host pages on the far socket crosses the
socket interconnect.  Prints one JSON line.

    python benchmarks/numa_probe.py [--bind local|none] [--reps 10]
"""
import argparse
import json
import os
import time


def gpu_locality(dev=0):
    import torch
    p = torch.cuda.get_device_properties(dev)
    bdf = "%04x:%02x:%02x.0" % (getattr(p, "pci_domain_id", 0), p.pci_bus_id, p.pci_device_id)
    base = "/sys/bus/pci/devices/" + bdf
    rd = lambda f: open(os.path.join(base, f)).read().strip() if os.path.exists(os.path.join(base, f)) else None
    return bdf, rd("numa_node"), rd("local_cpulist")


def parse_cpulist(s):
    out = []
    for part in s.split(","):
        if "-" in part:
            a, b = part.split("-")
            out += range(int(a), int(b) + 1)
        elif part:
            out.append(int(part))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bind", default="none", choices=["none", "local"])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--mb", type=int, default=131)
    a = ap.parse_args()
    import torch
    bdf, node, cpus = gpu_locality(0)
    before = sorted(os.sched_getaffinity(0))
    if a.bind == "local" and cpus:
        os.sched_setaffinity(0, parse_cpulist(cpus))
    dev = torch.device("cuda", 0)
    n = a.mb << 20
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    h.fill_(1)
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def timeit(fn):
        fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / a.reps

    h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
    d2 = torch.empty(n, dtype=torch.uint8, device=dev)

    def h2d():
        with torch.cuda.stream(s1):
            d.copy_(h, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)

    def both():
        h2d()
        d2h()

    print(json.dumps({"bind": a.bind, "gpu_bdf": bdf, "gpu_numa_node": node, "gpu_local_cpus": cpus,
                      "affinity_before": "%d cpus %d-%d" % (len(before), before[0], before[-1]),
                      "h2d_GBps": n / timeit(h2d) / 1e9, "d2h_GBps": n / timeit(d2h) / 1e9,
                      "both_GBps": 2 * n / timeit(both) / 1e9}))


if __name__ == "__main__":
    main()
