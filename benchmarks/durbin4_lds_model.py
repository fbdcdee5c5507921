#!/usr/bin/env python3
"""Bank model of durbin4_kernel's LDS relayouts (fdlp_lpc.hip c4_durbin), MI355X_MICROARCH.md "LDS":
ds_read_b64 / ds_write_b64 are served in two 32-lane groups, bank of double index d = (2 d) mod 64, so a
group is conflict-free iff its 32 lanes' d mod 32 are distinct; the extra cycles of a group = (largest
number of lanes on one d mod 32) - 1.

Lane = 4 ii + li (ii: item of the wave, li: lane in the item).  Item ii's image starts at kC4Guard + ii kItem;
a relayout of phase S writes img[li S + j] (j < S), reads R1n / An at img[li SN + j] (j < SN) and the mirrored
Bn at img[(4 S - 2) - li SN - j].  Prints, per phase and per access kind, the extra cycles per wave and
the total per launch (327 680 items = 20 480 waves), and the same for other item strides.

    python benchmarks/durbin4_lds_model.py
"""
import collections

GUARD, STEP, SL4 = 24, 4, 38


def item_stride(sl4):
    need = 4 * sl4
    return need + ((28 - need % 32) + 32) % 32


def extra(addrs):
    """extra LDS cycles of one wave-instruction (64 lane double indices), two 32-lane groups"""
    e = 0
    for g in (addrs[:32], addrs[32:]):
        c = collections.Counter(d % 32 for d in g)
        e += max(c.values()) - 1
    return e


def phases():
    s = 1
    while True:
        sn = min(s + STEP, SL4)
        yield s, sn
        if sn == s:
            return
        s = sn


def model(kitem):
    rows = []
    total = 0
    for s, sn in phases():
        base = [GUARD + (lane >> 2) * kitem for lane in range(64)]
        li = [lane & 3 for lane in range(64)]
        if sn == s:  # the last phase: gg, then A written once for the row copies
            w = sum(extra([base[x] + li[x] * s + j for x in range(64)]) for j in range(s))
            rows.append((s, sn, {"final_write": w}))
            total += w
            break
        k1c = 4 * s - 2
        wr = 2 * sum(extra([base[x] + li[x] * s + j for x in range(64)]) for j in range(s))  # R1 then A
        rd = 2 * sum(extra([base[x] + li[x] * sn + j for x in range(64)]) for j in range(sn))  # R1n, An
        rb = sum(extra([base[x] + k1c - li[x] * sn - j for x in range(64)]) for j in range(sn))  # Bn
        rows.append((s, sn, {"write": wr, "read": rd, "read_mirror": rb}))
        total += wr + rd + rb
    return rows, total


def main():
    kitem = item_stride(SL4)
    rows, total = model(kitem)
    waves = 327680 // 16
    print("item stride %d doubles (SL4 = %d)" % (kitem, SL4))
    for s, sn, d in rows:
        print("  phase S=%2d -> %2d  extra cycles per wave %s" % (s, sn, d))
    print("  total %d extra cycles per wave, %.3g per launch (%d waves)" % (total, total * waves, waves))
    best = sorted((model(k)[1], k) for k in range(4 * SL4 + 1, 4 * SL4 + 64))
    print("other strides (extra cycles per wave, stride):", best[:6])


if __name__ == "__main__":
    main()
