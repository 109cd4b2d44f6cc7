"""CPU model of the front's eval-window policies on JSON-slice values (round 6, PMC_EVAL_PRED).

Runs zlib deflate_slow (level 9: max_chain 4096, good 32, nice 258, lazy 258) on random slices of the
reference's tests/data corpus to get the positions the parse searches, then replays the front's evals:
an eval starts at the first searched position not yet evaluated and gives min(chain count, 32) lanes to
positions of its 64-position window until 64 lanes are used.  hops=0: every has-candidate position in order
(the round-5 front); hops=H: only the positions deflate_slow's walk visits when match lengths are the
nearest candidate's (capped at CAP), for H fresh starts, then the rest in order.  Diagnostic only.

usage: python scripts/eval_policy_sim.py VLEN SEED [N_VALUES] [CAP]
"""
import os, random, sys
D = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "data")
corpus = b"".join(open(os.path.join(D, f), "rb").read() for f in sorted(os.listdir(D)))
VLEN = int(sys.argv[1]); random.seed(int(sys.argv[2])); NV = int(sys.argv[3]) if len(sys.argv) > 3 else 150
CAP = int(sys.argv[4]) if len(sys.argv) > 4 else 32
def h3(b, p): return ((b[p] << 10) ^ (b[p + 1] << 5) ^ b[p + 2]) & 0x7fff
def mlen(b, p, q, n, cap=258):
    L = 0; m = min(cap, n - p)
    while L < m and b[p + L] == b[q + L]: L += 1
    return L
def run(b, hops_list):
    n = len(b); npos = n - 2; chains = {}; cand = []
    for p in range(npos):
        lst = chains.setdefault(h3(b, p), []); cand.append(lst[::-1][:4096]); lst.append(p)
    def longest(p, prev_len):
        chain = 1024 if prev_len >= 32 else 4096
        best, bs = 2, 0
        for i, q in enumerate(cand[p]):
            if i >= chain: break
            L = mlen(b, p, q, n)
            if L > best:
                best, bs = L, q
                if L >= 258 or L >= n - p: break
        if best == 3 and p - bs > 4096: best = 2
        return best
    full = []; s = 0; ml = 2
    while s < n:
        pl = ml; ml = 2
        if s < npos and cand[s] and pl < 258:
            full.append((s, pl)); ml = longest(s, pl)
        if pl >= 3 and ml <= pl: s += pl - 1; ml = 2
        else: s += 1
    L1 = [(mlen(b, p, cand[p][0], n, CAP) if cand[p] else 0) for p in range(npos)]
    res = {}
    for H in hops_list:
        ev = set(); nev = 0; npe = 0; nh = 0
        for (x, P) in full:
            if x in ev: continue
            nev += 1
            W = min(64, npos - x)
            hc = [1 if cand[x + l] else 0 for l in range(W)]
            mlv = [(L1[x + l] if L1[x + l] >= 3 else 2) if hc[l] else 2 for l in range(W)]
            imp = [mlv[l] > (mlv[l - 1] if l else P) for l in range(W)]
            inc = set([0])
            s = 0
            if H == 0:
                inc = set(range(W))
            else:
                if P >= 3 and not imp[0]:
                    s = P - 1
                hops = 0
                while s < W:
                    if hops >= H and H > 0:
                        inc |= set(range(s, W)); break
                    ms = [l for l in range(s, W) if hc[l]]
                    if not ms: break
                    s = ms[0]; inc.add(s); hops += 1; nh += 1
                    if mlv[s] < 3: s += 1; continue
                    t = s + 1
                    while t < W and imp[t]: t += 1
                    inc |= set(range(s, min(t + 1, W)))
                    if t >= W: break
                    s = t - 1 + mlv[t - 1]
            lanes = 0
            for l in range(W):
                if not hc[l] or l not in inc: continue
                c = min(len(cand[x + l]), 32)
                if lanes + c > 64: break
                lanes += c; ev.add(x + l); npe += 1
        res[H] = (nev, npe, len(full), nh)
    return res
tot = {}
HS = [0, 1, 2, 3, 4, 6, 99]
for i in range(NV):
    o = random.randrange(0, len(corpus) - VLEN)
    for k, v in run(corpus[o:o + VLEN], HS).items():
        t = tot.setdefault(k, [0] * 4)
        for j in range(4): t[j] += v[j]
for k, t in tot.items():
    print(f"hops<={k:2d}: evals/value {t[0]/NV:6.1f}  evaluated/value {t[1]/NV:6.1f}  searched {t[2]/NV:6.1f}  hops/eval {t[3]/max(t[0],1):.2f}")
