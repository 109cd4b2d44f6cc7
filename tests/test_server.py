"""The batched server on loopback: protocol semantics and pipelined load.

poor-man-s-cache_amd/pmc_codec/pmc_server gathers each epoll iteration's requests, runs the
iteration's compressions / decompressions as one device-store batch, and answers every connection
in request order.  The semantic checks mirror the reference server's custom protocol
(/root/reference/src/server/server.cpp:109-322, protocol.cpp:12-23): SET -> "OK", GET of a missing
key -> "(nil)", DEL of a missing key -> "ERROR: Key does not exist", malformed requests -> its error
strings; plus what batching must preserve: SET -> GET visibility and DEL inside one pipelined write,
and per-connection order.  pmc_loadgen then drives pipelined batches of 100 commands per connection
(tests/tcp_server_test.py -p -b 100 shape, BASELINE configs[4]) with 4 KiB JSON-slice values and
checks every GET against the last value SET.  CPU: --codec off (no device); GPU: the device store
(--codec batch) and the per-value drop-in path (--codec single).
"""
import json
import os
import socket
import subprocess
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "poor-man-s-cache_amd", "pmc_codec")
DATA = os.path.join(ROOT, "tests", "golden", "data")
SEP = b"\x1f"


@pytest.fixture(scope="module", autouse=True)
def _built():
    """pmc_server / pmc_loadgen are build outputs (not tracked): make them current before use."""
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "poor-man-s-cache_amd"), "pmc_codec/pmc_server",
                        "pmc_codec/pmc_loadgen"], capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        pytest.skip("pmc_server build failed: " + r.stderr[-500:])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Server:
    def __init__(self, codec, extra=()):
        self.port = _free_port()
        self.p = subprocess.Popen([os.path.join(BIN, "pmc_server"), "--port", str(self.port), "--codec", codec,
                                   "--heap-mb", "1024", *extra], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                  text=True)
        line = self.p.stdout.readline()
        assert line.startswith("READY"), (line, self.p.stderr.read() if self.p.poll() is not None else "")

    def stop(self):
        self.p.terminate()  # SIGTERM to this exact child: it prints its stats line and exits
        out, err = self.p.communicate(timeout=30)
        assert self.p.returncode == 0, err
        return json.loads(out.strip().splitlines()[-1])


def _exchange(port, cmds):
    """One pipelined write of all commands, then read len(cmds) responses.  The write waits 20 ms after the
    connect: the reference CacheServer adds a new fd to its epoll set before it records the connection
    (src/server/conn_manager.hpp:84-91) and reads that record without a lock (server.cpp:374, :408), so a
    request sent at once can be lost (test_ref_server.REF_CONNECT_RACE); pmc_server has no such window,
    and the delay costs it nothing.  A response missing for 60 s fails instead of hanging."""
    with socket.create_connection(("127.0.0.1", port)) as s:
        s.settimeout(60)
        time.sleep(0.02)
        s.sendall(SEP.join(cmds) + SEP)
        buf, out = b"", []
        while len(out) < len(cmds):
            while SEP not in buf:
                chunk = s.recv(1 << 16)
                assert chunk, "connection closed"
                buf += chunk
            r, buf = buf.split(SEP, 1)
            out.append(r)
        return out


def _semantics(port, golden, one_by_one=False):
    """one_by_one: every command in its own write, answered before the next is sent.  The reference
    server needs that when values are stored raw: a GET's response points at the stored value
    (kvs.cpp:224, server.cpp:115-116) and is sent after the whole epoll iteration (server.cpp:386-390),
    so a later SET of the same key in the same pipelined write frees it first (kvs.cpp:162) and the
    GET answers freed memory.  Compressed values are not affected (each GET gets its own buffer)."""
    big = golden.corpus[100:4196]        # compressed (strlen + 1 >= 30)
    big2 = golden.corpus[5000:9000]
    small = b"v" * 28                    # stored raw (strlen + 1 == 29)
    cmds = [b"GET nokey", b"SET a " + big, b"GET a", b"SET b " + small, b"GET b", b"SET a " + big2, b"GET a",
            b"DEL a", b"GET a", b"DEL a", b"SET c " + big + b" with spaces", b"GET c", b"BOGUS x",
            b"NOSPACE", b"SET k", b"GET "]
    want = [b"(nil)", b"OK", big, b"OK", small, b"OK", big2, b"OK", b"(nil)", b"ERROR: Key does not exist", b"OK",
            big + b" with spaces", b"ERROR: Unknown command", b"ERROR: Unable to parse request",
            b"ERROR: Invalid command format", b"ERROR: Invalid command format"]
    got = [r for c in cmds for r in _exchange(port, [c])] if one_by_one else _exchange(port, cmds)
    assert got == want
    # values committed by the batch above are served by later batches (the store, not the request)
    assert _exchange(port, [b"GET c", b"GET b", b"GET a"]) == [big + b" with spaces", small, b"(nil)"]
    # all the JSON files through the store, one batch each way
    files = [d for _, d in golden.data_files]
    assert _exchange(port, [b"SET f%d " % i + d for i, d in enumerate(files)]) == [b"OK"] * len(files)
    assert _exchange(port, [b"GET f%d" % i for i in range(len(files))]) == files


def _load(port, vlen, ops, conns=16, keys=8192, mix=50, proto="custom"):
    r = subprocess.run([os.path.join(BIN, "pmc_loadgen"), "--port", str(port), "--data", DATA, "--conns", str(conns),
                        "--keys", str(keys), "--vlen", str(vlen), "--ops", str(ops), "--batch", "100", "--mix",
                        str(mix), "--proto", proto], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["mismatches"] == 0 and res["failed_conns"] == 0, res
    return res


def test_server_semantics_and_load_without_codec(golden):
    s = Server("off")
    try:
        _semantics(s.port, golden)
        _load(s.port, 4096, 40_000)
    finally:
        st = s.stop()
    assert st["compressed"] == 0 and st["requests"] > 40_000


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["batch", "single"])
def test_server_on_gpu_codec(golden, codec):
    s = Server(codec)
    try:
        _semantics(s.port, golden)
        res = _load(s.port, 4096, 40_000 if codec == "batch" else 4_000)
    finally:
        st = s.stop()
    assert st["compressed"] > 8192 and st["decompressed"] > 0 and st["raw_fallbacks"] == 0, st
    if codec == "batch":
        assert st["pending_hits"] >= 1
    print(codec, res, st)


# ---- RESP (the reference's second protocol, server.cpp:147-280, protocol.cpp:294-567) ----------------------

def resp_cmd(*args):
    """A RESP array of bulk strings, as redis-py writes a command."""
    return b"*%d\r\n" % len(args) + b"".join(b"$%d\r\n%s\r\n" % (len(a), a) for a in args)


def _read_reply(s, buf):
    """One whole reply from buf (+recv): a RESP reply (+ - : $ *, arrays recursive) or a custom one (up to 0x1F,
    the separator kept).  -> (reply bytes, rest)."""
    def need(pred):
        nonlocal buf
        while True:
            k = pred(buf)
            if k is not None:
                return k
            chunk = s.recv(1 << 16)
            assert chunk, "connection closed"
            buf += chunk

    def line_end(at):
        return need(lambda b: (b.find(b"\r\n", at) + 2) if b.find(b"\r\n", at) >= 0 else None)

    def one(at):
        need(lambda b: at if len(b) > at else None)
        t = buf[at:at + 1]
        if t in (b"+", b"-", b":"):
            return line_end(at)
        if t == b"$":
            e = line_end(at)
            n = int(buf[at + 1:e - 2])
            return e if n < 0 else need(lambda b: e + n + 2 if len(b) >= e + n + 2 else None)
        if t == b"*":
            e = line_end(at)
            for _ in range(int(buf[at + 1:e - 2])):
                e = one(e)
            return e
        return need(lambda b: (b.find(SEP, at) + 1) if b.find(SEP, at) >= 0 else None)

    e = one(0)
    return buf[:e], buf[e:]


def resp_exchange(port, reqs, one_by_one=False):
    """reqs: encoded requests (RESP arrays, or custom ones ending in 0x1F) -> one reply each (bytes)."""
    with socket.create_connection(("127.0.0.1", port)) as s:
        s.settimeout(60)
        time.sleep(0.02)  # (see _exchange)
        out, buf = [], b""
        for chunk in ([[r] for r in reqs] if one_by_one else [reqs]):
            s.sendall(b"".join(chunk))
            for _ in chunk:
                r, buf = _read_reply(s, buf)
                out.append(r)
        return out


def _bulk(v):
    return b"$%d\r\n" % len(v) + v + b"\r\n"


def resp_semantics(port, golden, one_by_one=False):
    """GET/SET/DEL replies, MULTI/EXEC/DISCARD transactions and their errors, parse errors, and custom requests
    mixed into the same connection.  The replies are the reference server's own (test_ref_server checks that
    ref_server_zlib gives exactly these)."""
    big = golden.corpus[100:4196]
    big2 = golden.corpus[5000:9000]
    small = b"v" * 28
    R = resp_cmd
    pairs = [
        (R(b"GET", b"nokey"), b"$-1\r\n"),
        (R(b"SET", b"a", big), b"+OK\r\n"),
        (R(b"GET", b"a"), _bulk(big)),
        (R(b"SET", b"b", small), b"+OK\r\n"),
        (R(b"GET", b"b"), _bulk(small)),
        (R(b"SET", b"a", big2), b"+OK\r\n"),
        (R(b"GET", b"a"), _bulk(big2)),
        (b"GET a" + SEP, big2 + SEP),                       # a custom request on the same connection
        (R(b"DEL", b"a"), b":1\r\n"),
        (R(b"GET", b"a"), b"$-1\r\n"),
        (R(b"DEL", b"a"), b":0\r\n"),
        (R(b"MULTI"), b"+OK\r\n"),
        (R(b"SET", b"t", big), b"+QUEUED\r\n"),
        (R(b"GET", b"t"), b"+QUEUED\r\n"),
        (R(b"DEL", b"b"), b"+QUEUED\r\n"),
        (R(b"GET", b"b"), b"+QUEUED\r\n"),
        (R(b"EXEC"), b"*4\r\n+OK\r\n" + _bulk(big) + b":1\r\n$-1\r\n"),
        (R(b"EXEC"), b"-ERR ERR EXEC without MULTI\r\n"),
        (R(b"DISCARD"), b"-ERR ERR DISCARD without MULTI\r\n"),
        (R(b"MULTI"), b"+OK\r\n"),
        (R(b"MULTI"), b"-ERR ERR MULTI calls can not be nested\r\n"),
        (R(b"SET", b"x", big), b"+QUEUED\r\n"),
        (R(b"EXEC"), b"-ERR EXECABORT Transaction discarded because of previous errors.\r\n"),
        (R(b"GET", b"x"), b"$-1\r\n"),
        (R(b"MULTI"), b"+OK\r\n"),
        (R(b"SET", b"u", big2), b"+QUEUED\r\n"),
        (R(b"DISCARD"), b"+OK\r\n"),
        (R(b"GET", b"u"), b"$-1\r\n"),
        (R(b"MULTI"), b"+OK\r\n"),
        (R(b"EXEC"), b"*0\r\n"),
        (R(b"GET"), b"-ERR ERROR: Invalid command format\r\n"),
        (R(b"SET", b"k"), b"-ERR ERROR: Invalid command format\r\n"),
        (R(b"DEL", b"k", b"v"), b"-ERR ERROR: Invalid command format\r\n"),
        (R(b"get", b"t"), b"-ERR ERROR: Unknown command\r\n"),
        (b"*0\r\n", b"-ERR ERROR: Unable to parse request\r\n"),
        (R(b"SET", b"a", b"b", b"c"), b"-ERR ERROR: Unable to parse request\r\n"),
        (R(b"GET", b"t"), _bulk(big)),
        (R(b"SET", b"sp ace", big + b"\r\n\x1f*2\r\n"), b"+OK\r\n"),  # bulk bytes are not parsed
        (R(b"GET", b"sp ace"), _bulk(big + b"\r\n\x1f*2\r\n")),
    ]
    got = resp_exchange(port, [q for q, _ in pairs], one_by_one)
    bad = [(i, pairs[i][0][:40], got[i][:80], pairs[i][1][:80]) for i in range(len(pairs)) if got[i] != pairs[i][1]]
    assert not bad, bad
    # the JSON files through the store in RESP, one batch each way, and one EXEC reading them all
    files = [d for _, d in golden.data_files]
    assert resp_exchange(port, [R(b"SET", b"rf%d" % i, d) for i, d in enumerate(files)]) == [b"+OK\r\n"] * len(files)
    assert resp_exchange(port, [R(b"GET", b"rf%d" % i) for i in range(len(files))]) == [_bulk(d) for d in files]
    tx = [R(b"MULTI")] + [R(b"GET", b"rf%d" % i) for i in range(len(files))] + [R(b"EXEC")]
    got = resp_exchange(port, tx)
    assert got[-1] == b"*%d\r\n" % len(files) + b"".join(_bulk(d) for d in files)


def resp_malformed_closes(port):
    """A RESP array that cannot parse closes the connection, and requests framed from the same read are dropped
    unanswered (server.cpp:448-455)."""
    with socket.create_connection(("127.0.0.1", port)) as s:
        s.settimeout(30)
        time.sleep(0.02)
        s.sendall(resp_cmd(b"SET", b"dropped", b"x" * 40) + b"*2\r\n$x\r\n")
        assert s.recv(64) == b""
    assert resp_exchange(port, [resp_cmd(b"GET", b"dropped")]) == [b"$-1\r\n"]


def test_server_resp_without_codec(golden):
    s = Server("off")
    try:
        resp_semantics(s.port, golden)
        resp_malformed_closes(s.port)
        _load(s.port, 4096, 20_000, proto="resp")
    finally:
        st = s.stop()
    assert st["resp_requests"] > 20_000


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["batch", "single"])
def test_server_resp_on_gpu_codec(golden, codec):
    """Stored values answer RESP GETs as bulk strings framed on the device (PMC_FRAME_RESP) in the same store
    batch as custom GETs (pmc_store_get_batch_frames)."""
    s = Server(codec)
    try:
        resp_semantics(s.port, golden)
        resp_malformed_closes(s.port)
        _semantics(s.port, golden)
        res = _load(s.port, 4096, 40_000 if codec == "batch" else 4_000, keys=8192 if codec == "batch" else 1024,
                    proto="resp")
    finally:
        st = s.stop()
    print(codec, res, st)
    assert st["compressed"] > 1000 and st["decompressed"] > 20 and st["raw_fallbacks"] == 0, st
