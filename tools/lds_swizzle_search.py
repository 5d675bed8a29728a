"""Search for an XOR-linear LDS swizzle for the float64 FFT of mss_target_kernel (dev tool).

Models every LDS access of its Stockham stages and post-twist at n = 64 .. 2048 against the
ds_read_b128 / ds_write_b128 bank rules of MI355X_MICROARCH.md and counts conflict cycles;
greedy + random-restart local search over swizzles i ^ h(bits 3..10 of i).

  python tools/lds_swizzle_search.py          # round-5 schedule: load pass + radix-4 stages
  python tools/lds_swizzle_search.py radix8   # round 6: first stage in registers, then radix 8
                                              # (remainder 2 / 4; radix 16 first at n = 2048)"""
import itertools, random
import numpy as np
G128R = [list(range(0,4))+list(range(12,16))+list(range(20,28)),
         list(range(4,12))+list(range(16,20))+list(range(28,32))]
G128R = G128R + [[l+32 for l in g] for g in G128R]
def conflicts_read(elems, phys):  # ds_read_b128: 16 B elems, 16 slots per bank row
    c = 0
    for g in G128R:
        slots = [phys[elems[l]] % 16 for l in g]
        cnt = np.bincount(slots, minlength=16)
        c += cnt.max() - 1
    return c
def conflicts_write(elems, phys):  # ds_write_b128: 8 x 8 contiguous, 8 slots per 128 B row
    c = 0
    for g0 in range(0, 64, 8):
        slots = [phys[elems[l]] % 8 for l in range(g0, g0+8)]
        cnt = np.bincount(slots, minlength=8)
        c += cnt.max() - 1
    return c
def patterns(LOG2M, BWT):
    """LDS accesses of wave_fft_d<LOG2M, BWT> + load + post-twist: list of (kind, elems[64])"""
    N = 1 << LOG2M; NR = N // 4; IT = BWT // 4 // 64
    acc = []
    # load/window store S[e], e = lane + 64 kk
    for kk in range(BWT // 64):
        acc.append(('w', [l + 64*kk for l in range(64)]))
    Ns = 1
    for st in range(LOG2M // 2):
        for it in range(IT):
            idx = [l + 64*it for l in range(64)]
            for r in range(4):
                acc.append(('r', [ (i//NR)*N + (i%NR) + r*NR for i in idx]))
        for it in range(IT):
            idx = [l + 64*it for l in range(64)]
            for r in range(4):
                el = []
                for i in idx:
                    fr, j = i//NR, i%NR; k = j % Ns
                    el.append(fr*N + (j-k)*4 + k + r*Ns)
                acc.append(('w', el))
        Ns *= 4
    if LOG2M & 1:
        NR2 = N//2; IT2 = BWT//2//64
        for it in range(IT2):
            idx = [l + 64*it for l in range(64)]
            acc.append(('r', [(i//NR2)*N + i%NR2 for i in idx]))
            acc.append(('r', [(i//NR2)*N + i%NR2 + NR2 for i in idx]))
        for it in range(IT2):
            idx = [l + 64*it for l in range(64)]
            el0, el1 = [], []
            for i in idx:
                fr, j = i//NR2, i%NR2; k = j % Ns
                el0.append(fr*N + (j-k)*2 + k); el1.append(fr*N + (j-k)*2 + k + Ns)
            acc.append(('w', el0)); acc.append(('w', el1))
    # post-twist: HALF = N complex per frame, NBIN = N+1 bins, FBT = BWT/N frames
    FBT = BWT // N; NBIN = N + 1
    NEO = (FBT*NBIN + 63)//64
    for jj in range(NEO):
        a, b = [], []
        for l in range(64):
            e = l + 64*jj
            e = min(e, FBT*NBIN-1)
            m, f = e // NBIN, e % NBIN
            a.append(m*N + (f & (N-1))); b.append(m*N + ((N - f) & (N-1)))
        acc.append(('r', a)); acc.append(('r', b))
    return acc
def cost(phys, pats):
    return sum(conflicts_read(e, phys) if k=='r' else conflicts_write(e, phys) for k, e in pats)
def mkphys(vecs, size):
    i = np.arange(size)
    h = np.zeros(size, dtype=int)
    for b, v in vecs.items():
        h ^= ((i >> b) & 1) * v
    return i ^ h
def sched8(L, BWT):
    if L == 10 and BWT >= 1024:
        return [16, 8, 8]
    a, b = divmod(L, 3)
    return [8] * a + ([2 ** b] if b else [])
def patterns_radix8(LOG2M, BWT):
    """the round-6 schedule: the first stage's inputs come from registers (no load pass)"""
    N = 1 << LOG2M; acc = []; Ns = 1
    for si, R in enumerate(sched8(LOG2M, BWT)):
        NR = N // R; IT = BWT // R // 64
        if si > 0:
            for it in range(IT):
                idx = [l + 64*it for l in range(64)]
                for r in range(R):
                    acc.append(('r', [(i//NR)*N + i%NR + r*NR for i in idx]))
        for it in range(IT):
            idx = [l + 64*it for l in range(64)]
            for r in range(R):
                el = []
                for i in idx:
                    fr, j = i//NR, i%NR; k = j % Ns
                    el.append(fr*N + (j-k)*R + k + r*Ns)
                acc.append(('w', el))
        Ns *= R
    acc += [a for a in patterns(LOG2M, BWT) if a[0] == 'r'][-2 * ((BWT // N * (N + 1) + 63) // 64):]
    return acc
import sys
configs = [(5,512),(6,512),(7,512),(8,512),(9,512),(10,1024)]
gen = patterns_radix8 if sys.argv[1:] == ['radix8'] else patterns
allp = {c: gen(*c) for c in configs}
ident = {c: cost(np.arange(c[1]), allp[c]) for c in configs}
print("identity", ident, sum(ident.values()))
best = None
random.seed(0)
bits = list(range(3, 10))
def total(vecs):
    return sum(cost(mkphys(vecs, c[1]), allp[c]) for c in configs)
cur = {}
curc = total(cur)
for rnd in range(3):
    for b in bits:
        bestv, bestc = cur.get(b, 0), curc
        for v in range(16):
            if b == 3 and v >= 8: continue
            t = dict(cur); t[b] = v
            if (v >> 0) and b < 4 and (v & (1 << b)) == 0: pass
            c = total(t)
            if c < bestc: bestv, bestc = v, c
        cur[b] = bestv; curc = bestc
    print(rnd, cur, curc)
print("per size", {c: cost(mkphys(cur, c[1]), allp[c]) for c in configs})
bits = list(range(3, 11))
bestall = (curc, dict(cur))
for start in range(12):
    cur = {b: (random.randrange(8) if b == 3 else random.randrange(16)) for b in bits}
    curc = total(cur)
    improved = True
    while improved:
        improved = False
        for b in bits:
            for v in range(8 if b == 3 else 16):
                if v == cur[b]: continue
                t = dict(cur); t[b] = v
                c = total(t)
                if c < curc:
                    cur, curc, improved = t, c, True
    if curc < bestall[0]:
        bestall = (curc, dict(cur))
    print(start, curc, cur, flush=True)
print("BEST", bestall)
print("per size", {c: cost(mkphys(bestall[1], c[1]), allp[c]) for c in configs})
