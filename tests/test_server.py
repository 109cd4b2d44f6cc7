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


def _load(port, vlen, ops, conns=16, keys=8192, mix=50):
    r = subprocess.run([os.path.join(BIN, "pmc_loadgen"), "--port", str(port), "--data", DATA, "--conns", str(conns),
                        "--keys", str(keys), "--vlen", str(vlen), "--ops", str(ops), "--batch", "100", "--mix",
                        str(mix)], capture_output=True, text=True, timeout=240)
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
