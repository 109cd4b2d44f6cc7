"""Test helper: dissect a gzip member into blocks / code lengths / tokens (pure Python).

Used to explain a parity failure: diff(dissect(gpu_bytes), dissect(golden_bytes)) says
whether the parse (tokens), the Huffman trees (code lengths) or the bit emission differs.
"""

LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163,
         195, 227, 258]
LEXT = [0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
         4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]
ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


class Bits:
    def __init__(self, data, pos=0):
        self.d, self.p = data, pos * 8

    def get(self, n):
        v = 0
        for k in range(n):
            b = self.p + k
            v |= ((self.d[b >> 3] >> (b & 7)) & 1) << k
        self.p += n
        return v


def _decoder(lens):
    codes, code, nxt = {}, 0, {}
    bl = [0] * 16
    for x in lens:
        if x:
            bl[x] += 1
    for L in range(1, 16):
        code = (code + bl[L - 1]) << 1
        nxt[L] = code
    for s, L in enumerate(lens):
        if L:
            codes[(L, nxt[L])] = s
            nxt[L] += 1
    return codes


def _sym(br, dec):
    code = 0
    for L in range(1, 16):
        code = (code << 1) | br.get(1)
        if (L, code) in dec:
            return dec[(L, code)]
    raise ValueError("bad code")


def dissect(gz: bytes):
    br = Bits(gz, 10)
    blocks = []
    while True:
        last, typ = br.get(1), br.get(2)
        blk = {"type": typ, "last": last, "start_bit": br.p - 3}
        if typ == 0:
            br.p = (br.p + 7) & ~7
            n = br.get(16)
            br.get(16)
            br.p += 8 * n
            blk["stored_len"] = n
        else:
            if typ == 1:
                ll = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
                dl = [5] * 30
            else:
                hlit, hdist, hclen = br.get(5) + 257, br.get(5) + 1, br.get(4) + 4
                cl = [0] * 19
                for k in range(hclen):
                    cl[ORDER[k]] = br.get(3)
                cdec = _decoder(cl)
                lens = []
                while len(lens) < hlit + hdist:
                    s = _sym(br, cdec)
                    if s < 16:
                        lens.append(s)
                    elif s == 16:
                        lens += [lens[-1]] * (3 + br.get(2))
                    elif s == 17:
                        lens += [0] * (3 + br.get(3))
                    else:
                        lens += [0] * (11 + br.get(7))
                ll, dl = lens[:hlit], lens[hlit:]
                blk.update(hlit=hlit, hdist=hdist, hclen=hclen, cl=cl, tree_end_bit=br.p)
            blk["ll"], blk["dl"] = ll, dl
            ld, dd = _decoder(ll), _decoder(dl)
            toks = []
            while True:
                s = _sym(br, ld)
                if s < 256:
                    toks.append(s)
                elif s == 256:
                    break
                else:
                    s -= 257
                    ln = LBASE[s] + br.get(LEXT[s])
                    d = _sym(br, dd)
                    dist = DBASE[d] + br.get(DEXT[d])
                    toks.append((ln, dist))
            blk["tokens"] = toks
        blocks.append(blk)
        if last:
            break
    return blocks


def explain(got: bytes, want: bytes) -> str:
    """One-line verdict on where two gzip members diverge."""
    first = next((k for k in range(min(len(got), len(want))) if got[k] != want[k]), min(len(got), len(want)))
    msg = [f"len {len(got)} vs {len(want)}, first diff at byte {first}"]
    try:
        g, w = dissect(got), dissect(want)
    except Exception as e:  # noqa: BLE001
        return "; ".join(msg + [f"dissect failed: {e!r}"])
    if len(g) != len(w):
        return "; ".join(msg + [f"blocks {len(g)} vs {len(w)}"])
    for i, (a, b) in enumerate(zip(g, w)):
        if a["type"] != b["type"]:
            msg.append(f"block {i} type {a['type']} vs {b['type']}")
            break
        if a.get("tokens") != b.get("tokens"):
            ta, tb = a.get("tokens", []), b.get("tokens", [])
            k = next((j for j in range(min(len(ta), len(tb))) if ta[j] != tb[j]), min(len(ta), len(tb)))
            msg.append(f"block {i} tokens differ at #{k}: {ta[k:k + 3]} vs {tb[k:k + 3]}")
            break
        for key in ("hlit", "hdist", "hclen", "cl", "ll", "dl"):
            if a.get(key) != b.get(key):
                msg.append(f"block {i} {key} differs")
                break
        else:
            msg.append(f"block {i} structures equal (bit emission differs)")
    return "; ".join(msg)
