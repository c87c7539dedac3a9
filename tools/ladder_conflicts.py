#!/usr/bin/env python3
"""Host count of the fused ladder's LDS read cycles:
every cfg2 rung (f = 0.1 / (256 us x 240) x (261/240)^k, 57 rungs) over one
3584-sample span, its outputs in waves of 64 consecutive outputs (two 32-lane
groups per ds_read), each read instruction j of the window (window start
floor(k f) + j) priced as the largest number of distinct addresses on one
bank in a group (ds_read_b32: 32 banks; identical addresses broadcast).
Layouts: plain, a pad word every 32 / 64 floats, XOR bank swizzle; and
8-byte aligned pairs (ds_read_b64, 64 banks).  CPU only.

usage: python tools/ladder_conflicts.py [plain pad32 pad64 xor pad32x3]
"""
import math
import sys

f0 = 0.1/(256e-6*240); g = 261/240
rungs = [f0*g**k for k in range(57)]
SPAN = 3584
def cycles(addrs, nb=32):
    # addrs: [64] lane addresses (None = inactive); ds_read_b32: two 32-lane groups
    tot = 0
    for h in (0, 32):
        a = [x for x in addrs[h:h+32] if x is not None]
        if not a: continue
        banks = {}
        for x in set(a):
            banks.setdefault(x % nb, set()).add(x)
        tot += max(len(v) for v in banks.values())
    return tot
def layout(i, kind):
    if kind == 'plain': return i
    if kind == 'pad32': return i + (i >> 5)
    if kind == 'pad64': return i + (i >> 6)
    if kind == 'xor': return (i & ~31) | ((i ^ (i >> 5)) & 31)
    if kind == 'pad32x3': return i + 3*(i >> 5)
    raise
def sim(kind, s0=0):
    res = {}
    for f in rungs:
        klo = math.ceil(s0/f); khi = math.ceil((s0+SPAN)/f)
        ks = list(range(klo, khi))
        CC = int(f) + 1
        nread = CC if CC <= 12 else None
        tot = 0; ideal = 0
        for w0 in range(0, len(ks), 64):
            lanes = ks[w0:w0+64]
            starts = [int(math.floor(k*f)) - s0 for k in lanes]
            cnt = [int(math.floor(k*f+f)) - int(math.floor(k*f)) for k in lanes]
            nr = CC if CC <= 12 else 1 + 8*math.ceil((max(cnt)-1)/8) + 1
            for j in range(nr):
                ad = [layout(st + j, kind) for st in starts] + [None]*(64-len(starts))
                tot += cycles(ad); ideal += (1 if len(starts) <= 32 else 2)
        res[f] = (tot, ideal)
    return res
for kind in sys.argv[1:]:
    r = sim(kind)
    T = sum(v[0] for v in r.values()); I = sum(v[1] for v in r.values())
    small = sum(v[0] for f, v in r.items() if f < 11); smallI = sum(v[1] for f, v in r.items() if f < 11)
    print(kind, "cycles", T, "ideal", I, "ratio %.2f" % (T/I), "f<11: %.2f" % (small/smallI), "f>=11: %.2f" % ((T-small)/(I-smallI)))

def cycles_b64(addrs):
    # ds_read_b64: 2 x 32-lane groups, bank of dword address a = a mod 64, each lane 2 dwords
    tot = 0
    for h in (0, 32):
        a = [x for x in addrs[h:h+32] if x is not None]
        if not a: continue
        banks = {}
        for x in set(a):
            for d in (x, x+1):
                banks.setdefault(d % 64, set()).add(x)
        tot += 2 * max(len(v) for v in banks.values())   # 2 LDS cycles per wave instr when conflict-free -> per group 1? use 2 per instr total
    return tot / 2 * 1  # normalise: conflict-free instr = 2 cycles (1 per group)
def sim_b64():
    T = I = 0
    Ts = Is = 0
    for f in rungs:
        ks = list(range(0, math.ceil(SPAN/f)))
        CC = int(f) + 1
        for w0 in range(0, len(ks), 64):
            lanes = ks[w0:w0+64]
            starts = [int(math.floor(k*f)) for k in lanes]
            cnt = [int(math.floor(k*f+f)) - int(math.floor(k*f)) for k in lanes]
            ncols = CC if CC <= 12 else max(cnt) + 1
            npair = (ncols + 1 + 1) // 2
            for j in range(npair):
                ad = [2*(st//2) + 2*j for st in starts] + [None]*(64-len(starts))
                c = cycles_b64(ad)
                T += c; I += (1 if len(starts) <= 32 else 2)
                if f < 11: Ts += c; Is += (1 if len(starts) <= 32 else 2)
    print("b64 cycles", T, "f<11 cycles", Ts, "f>=11", T-Ts)
def sim_b32_total():
    T = 0; Ts = 0
    for f in rungs:
        ks = list(range(0, math.ceil(SPAN/f)))
        CC = int(f) + 1
        for w0 in range(0, len(ks), 64):
            lanes = ks[w0:w0+64]
            starts = [int(math.floor(k*f)) for k in lanes]
            cnt = [int(math.floor(k*f+f)) - int(math.floor(k*f)) for k in lanes]
            ncols = CC if CC <= 12 else 1 + 8*math.ceil((max(cnt)-1)/8) + 1
            for j in range(ncols):
                c = cycles([st + j for st in starts] + [None]*(64-len(starts)))
                T += c
                if f < 11: Ts += c
    print("b32 cycles", T, "f<11 cycles", Ts, "f>=11", T-Ts)
sim_b32_total(); sim_b64()
