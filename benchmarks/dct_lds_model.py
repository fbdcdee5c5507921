#!/usr/bin/env python3
"""LDS bank model of dct_frame_kernel (csrc/fdlp_dct.hip): every LDS access of one frame's workgroup
(640 threads = 10 waves), its lanes' addresses and the bank rules of MI355X_MICROARCH.md §LDS (lane groups
per instruction, (a/4) mod 64 or mod 32 banks, one extra cycle per extra distinct address on a bank).
Prints the extra (conflict) cycles per frame by access site, for the layout in the kernel, so that a
padding / table layout can be chosen on the CPU and then confirmed with SQ_LDS_BANK_CONFLICT.

    python3 benchmarks/dct_lds_model.py            # the kernel's layout
"""
import collections
import sys

A, B, C = 20, 24, 25
M = A * B * C
BC, AC, AB = B * C, A * C, A * B
THREADS = 640

GROUPS = {  # lane groups per instruction and the bank modulus (in dwords)
    "read_b64": ([list(range(0, 32)), list(range(32, 64))], 64, 2),
    "read_b128": ([[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)],
                   [*range(32, 36), *range(44, 48), *range(52, 60)], [*range(36, 44), *range(48, 52), *range(60, 64)]],
                  64, 4),
    "write_b64": ([list(range(g, g + 16)) for g in range(0, 64, 16)], 32, 2),
    "read2_b64": ([list(range(g, g + 16)) for g in range(0, 64, 16)], 32, 2),  # per access
}


def extra_cycles(kind, addr):
    """addr: {lane: byte address} of one wave-instruction (active lanes only) -> extra LDS cycles."""
    groups, nb, dw = GROUPS[kind]
    extra = 0
    for g in groups:
        banks = collections.defaultdict(set)
        for ln in g:
            if ln in addr:
                for d in range(dw):
                    w = addr[ln] // 4 + d
                    banks[w % nb].add(w)
        if banks:
            extra += max(len(v) for v in banks.values()) - 1
    return extra


def wave_instr(kind, f, lanes_of_thread, tot, site):
    """f(t) -> byte address or None (inactive) for the threads of each wave; accumulate per site."""
    for w in range(THREADS // 64):
        addr = {}
        for ln in range(64):
            t = 64 * w + ln
            a = f(t)
            if a is not None:
                addr[ln] = a
        if addr:
            tot[site] += extra_cycles(kind, addr)


def pass3_task(t):
    p, s = t >> 1, t & 1
    if p < 9 * B:
        a, b = 1 + p % 9, p // 9
        return (A - a if s else a), (B - 1 - b if s else b)
    if p < 9 * B + B // 2:
        b = p - 9 * B
        return A // 2, (B - 1 - b if s else b)
    if p < 9 * B + B - 1:
        b = p - (9 * B + B // 2) + 1
        return 0, (B - b if s else b)
    return 0, (B // 2 if s else 0)


def model(lay):
    """lay: layout functions (double indices).  Returns {site: extra cycles per frame}."""
    tot = collections.Counter()
    tw = lay["tw1"]
    for k1 in range(1, A):  # pass-1 twiddle: two double2 table reads per k1
        for which in (0, 1):
            wave_instr("read_b128", lambda t: (16 * tw(k1, t, which)) if t < BC else None, None, tot, "tw1")
    for h in range(2):
        for k1 in range(A):  # exchange 1 writes
            wave_instr("write_b64", lambda t: 8 * lay["x1"](k1, t) if t < BC else None, None, tot, "x1_w")
        for q2 in range(B):  # exchange 1 reads
            wave_instr(lay.get("x1_rkind", "read_b64"),
                       lambda t: 8 * lay["x1"](t // C, C * q2 + t % C) if t < AC else None, None, tot, "x1_r")
    for k2a in range(1, B):  # pass-2 twiddle
        wave_instr("read_b128", lambda t: 16 * lay["tw2"](k2a, t % C) if t < AC else None, None, tot, "tw2")
    for h in range(2):
        for j in range(B):  # exchange 2 writes: pass-2 thread (k1b, q3) value k2a = j
            wave_instr("write_b64", lambda t: 8 * lay["x2"](j, t // C, t % C) if t < AC else None, None, tot, "x2_w")
        for j in range(C):  # exchange 2 reads: pass-3 task (k1, k2a) value q3 = j
            def rd(t):
                if t >= AB:
                    return None
                k1, k2a = pass3_task(t)
                return 8 * lay["x2"](k2a, k1, j)
            wave_instr(lay.get("x2_rkind", "read_b64"), rd, None, tot, "x2_r")
    for half in range(2):  # D staging writes (D[k] for k = lo + AB j), then coalesced row reads
        for j in range(C):
            def wr(t):
                if t >= AB:
                    return None
                k1, k2a = pass3_task(t)
                if k1 == 0 and k2a == 0:
                    return None  # task (0, 0): the helper lanes write it
                return 8 * lay["d"](k1 + A * k2a + AB * j)
            wave_instr("write_b64", wr, None, tot, "d_w")
        for it in range((M // 2 + THREADS - 1) // THREADS):
            wave_instr("read_b128", lambda t: (8 * lay["d"](2 * (t + THREADS * it))
                                               if t + THREADS * it < M // 2 else None), None, tot, "d_r")
    return tot


def kernel_layout():
    kTwM, kTwA = 0, BC

    def tw1(k1, t, which):
        e = k1 * t
        a, b = e // BC, e % BC
        return kTwA + a if which == 0 else kTwM + b
    return {"tw1": tw1,
            "x1": lambda k1, n2: k1 * BC + n2,
            "tw2": lambda k2a, q3: BC + A + k2a * q3,
            "x2": lambda k2a, k1, q3: k2a * AC + k1 * C + q3,
            "d": lambda k: k}


def report(name, tot):
    print("%-28s total %7d   " % (name, sum(tot.values())) + "  ".join("%s %d" % kv for kv in sorted(tot.items())))


def new_layout(q1=601, p1=25, p2=500, dpad=None):
    """Conflict-free twiddle tables (pass 1: W_M^{k1 (t mod 16)} x W_M^{16 k1 (t div 16)}; pass 2:
    W_BC^{k2a q3} stored [k2a][q3]) and padded exchange images."""
    def tw1(k1, t, which):
        return (k1 * 16 + t % 16) if which == 0 else (A * 16 + k1 * 38 + t // 16)
    d = (lambda k: k) if dpad is None else dpad
    return {"tw1": tw1,
            "x1": lambda k1, n2: k1 * q1 + n2,
            "tw2": lambda k2a, q3: k2a * C + q3,
            "x2": lambda k2a, k1, q3: k2a * p2 + k1 * p1 + q3,
            "d": d}


if __name__ == "__main__":
    report("kernel (r03)", model(kernel_layout()))
    report("new tables, q1 601", model(new_layout()))
    best = []
    for p1 in range(25, 34):
        for p2 in range(max(500, 20 * p1), 20 * p1 + 40):
            t = model(dict(new_layout(p1=p1, p2=p2)))
            best.append((t["x2_r"] + t["x2_w"], p1, p2))
    best.sort()
    print("x2 layouts (conflicts, p1, p2):", best[:8])
    bd = []
    for P in range(16, 512, 2):
        for dlt in (2, 4, 6, 8):
            t = model(new_layout(dpad=lambda k, P=P, dlt=dlt: k + dlt * (k // P)))
            bd.append((t["d_w"] + t["d_r"], P, dlt))
    bd.sort()
    print("d layouts (conflicts, P, delta):", bd[:8])
    sys.exit(0)
