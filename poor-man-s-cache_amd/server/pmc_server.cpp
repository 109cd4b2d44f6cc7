// pmc_server.cpp -- a batched cache server over the GPU codec (with f2/f3/e).
//
// The reference server (/root/reference/src/server/server.cpp) runs one request thread: each epoll
// iteration reads every ready connection, then processes the pending requests one by one
// (handleRequests, server.cpp:361-384), each SET/GET calling the codec for ONE value
// (kvs.cpp:183,233), and finally sends each connection's responses with one sendmsg
// (server.cpp:386-390, 541-601).  That iteration is the batch boundary this server uses:
//   1. read every ready connection and frame its custom-protocol requests on 0x1F
//      (readRequestAsync, server.cpp:402-490);
//   2. apply the iteration's requests IN ORDER to the host key index -- SET/GET/DEL semantics of
//      processRequestSync (server.cpp:109-322) and KeyValueStore (kvs.cpp:141-235): a value is
//      compressed iff compression is on and strlen + 1 >= 30 (kvs.hpp:26, kvs.cpp:182); a GET that
//      follows a SET of the same key in the iteration answers with that SET's value (no codec);
//   3. run the iteration's compressions as ONE pmc_store_put_batch per GPU (values go to HBM
//      extents, f2) and its decompressions of stored values as ONE pmc_store_get_batch_frames per GPU,
//      framed as value + 0x1F or a RESP bulk string straight into a pinned send image (f3); GPUs run on their own threads
//      (shard = hashFunc(key) % shards, GPU = shard % nGPU: server.cpp:113,121,132 and SURVEY §8e);
//   4. send each connection's responses in request order with one sendmsg (iovecs point into the
//      pinned image, the request buffers and static strings: no value is copied on the host).
// A failed compression stores the raw value (kvs.cpp:188-192); extents replaced or deleted during
// an iteration are released after its GETs ran.  --codec single instead calls the single-value
// C-ABI (what the unchanged server does through the drop-in GzipCompressor), --codec off stores
// raw values (ENABLE_COMPRESSION=false).
// Both of the reference's protocols: custom requests end at 0x1F; RESP arrays ("*<n>\r\n" + bulk strings,
// GET/SET/DEL and MULTI/EXEC/DISCARD transactions, server.cpp:147-280) are framed by their lengths
// (protocol.cpp:294-356) and answered as RESP (protocol.cpp:399-567): a stored value's bulk string
// "$<len>\r\n<value>\r\n" is framed in the same device batch as the custom GETs (per-extent frames).
//
// usage: pmc_server --port P [--gpus N] [--shards 128] [--codec batch|single|off] [--heap-mb M]
//        prints "READY <port>" once listening; SIGTERM/SIGINT -> one JSON stats line, exit 0.
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "pmc_codec.h"

namespace {

constexpr char kSep = 0x1F;                     // MSG_SEPARATOR (protocol.hpp:17)
constexpr size_t kMinCompress = 30;             // MIN_SIZE_TO_COMPRESS (kvs.hpp:26), vs strlen + 1
const char kOK[] = "OK";                        // protocol.cpp:12-20
const char kNil[] = "(nil)";
const char kKeyNotExists[] = "ERROR: Key does not exist";
const char kInternal[] = "ERROR: Internal error";
const char kUnknown[] = "ERROR: Unknown command";
const char kUnparsable[] = "ERROR: Unable to parse request";
const char kBadFormat[] = "ERROR: Invalid command format";
// RESP payloads (protocol.cpp:36-48, protocol.hpp:24-25): errors are "-ERR " + message + CRLF
const char kRespOK[] = "+OK\r\n";
const char kRespQueued[] = "+QUEUED\r\n";
const char kRespNil[] = "$-1\r\n";
const char kRespOne[] = ":1\r\n";
const char kRespZero[] = ":0\r\n";
const char kRespErrNested[] = "-ERR ERR MULTI calls can not be nested\r\n";
const char kRespErrExecNoMulti[] = "-ERR ERR EXEC without MULTI\r\n";
const char kRespErrDiscardNoMulti[] = "-ERR ERR DISCARD without MULTI\r\n";
const char kRespErrExecAborted[] = "-ERR EXECABORT Transaction discarded because of previous errors.\r\n";
const char kRespErrUnknown[] = "-ERR ERROR: Unknown command\r\n";
const char kRespErrUnparsable[] = "-ERR ERROR: Unable to parse request\r\n";
const char kRespErrBadFormat[] = "-ERR ERROR: Invalid command format\r\n";

volatile sig_atomic_t g_stop = 0;
void on_signal(int) { g_stop = 1; }

enum class Codec { kBatch, kSingle, kOff };

enum : uint8_t { kCustom = 0, kResp = 1 };
enum : uint8_t { kGet, kSet, kDel };
struct TxCmd {  // a command queued by MULTI (RespTransactionState, persisted strings: server.cpp:161-173)
    uint8_t type;
    std::string key, val;
};

struct Conn {
    int fd = -1;
    std::string in;     // received bytes; requests of this iteration point into it
    size_t parsed = 0;  // bytes framed into requests so far
    std::string out;    // response bytes a previous sendmsg could not take
    bool closing = false;
    bool tx_active = false, tx_aborted = false;  // RESP MULTI state (server.cpp:148-159)
    std::vector<TxCmd> tx;
};

enum : uint8_t { kRaw = 0, kDevice = 1, kHostGz = 2, kPending = 3 };
struct Entry {
    uint8_t kind = kRaw;
    uint32_t gpu = 0;
    uint32_t put = 0;    // kPending: index in the iteration's put list of that GPU
    std::string bytes;   // kRaw: the value; kHostGz: its gzip member
    pmc_extent ext{};    // kDevice
};

// a response: static text, bytes of the arena, a pending SET value, or a store GET result
enum : uint8_t { kStatic, kArena, kView, kStoreGet };
struct Resp {
    uint8_t kind = kStatic;
    uint8_t proto = kCustom;  // kCustom: + 0x1F on the wire; kResp: the bytes are the whole RESP reply
    uint32_t gpu = 0;
    const char *p = nullptr;  // kStatic / kView
    size_t off = 0, n = 0;    // kArena: offset + length; kStoreGet: index in gets[gpu]
};
struct Req {
    Conn *c;
    Resp r;
};

struct Put {
    std::string_view key, val;
};

struct Gpu {
    pmc_ctx *ctx = nullptr;
    pmc_store *store = nullptr;
    std::vector<Put> puts;
    std::vector<pmc_extent> put_ext, gets, to_free;
    std::vector<uint8_t> get_frame;  // PMC_FRAME_CUSTOM / PMC_FRAME_RESP per get
    std::vector<int32_t> put_rc, get_rc;
    std::vector<const uint8_t *> get_resp;
    std::vector<uint32_t> get_len;
    int err = 0;
};

struct Stats {
    uint64_t iterations = 0, requests = 0, resp_requests = 0, sets = 0, gets = 0, dels = 0, compressed = 0, decompressed = 0,
             raw_fallbacks = 0, pending_hits = 0, put_calls = 0, get_calls = 0;
    double t_codec = 0, t_put = 0, t_get = 0, t_iter = 0;  // seconds: codec phase, store calls, whole iterations
};
double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

class Server {
  public:
    Codec codec = Codec::kBatch;
    uint32_t shards = 128;
    std::vector<Gpu> gpus;
    std::vector<std::unordered_map<std::string, Entry>> index;
    Stats st;

    int run(int port);

  private:
    int ep = -1, lfd = -1;
    std::unordered_map<int, std::unique_ptr<Conn>> conns;
    std::vector<Req> reqs;
    std::string arena;
    std::vector<std::vector<TxCmd>> tx_keep;  // EXEC'd queues: puts and views point into them this iteration

    void accept_all();
    void read_conn(Conn *c);
    void frame(Conn *c);
    void process();
    void apply(size_t q, std::string_view payload);
    void apply_resp(Conn *c, size_t q, std::string_view payload);
    void do_set(Resp &r, std::string_view key, std::string_view val);
    void do_get(Resp &r, std::string_view key);
    void do_del(Resp &r, std::string_view key);
    size_t push_req(Conn *c, uint8_t proto) {
        reqs.push_back(Req{c, Resp{}});
        reqs.back().r.proto = proto;
        return reqs.size() - 1;
    }
    void resp_bulk_arena(Resp &r, const char *p, size_t n);
    void run_codec();
    void send_conn(Conn *c, size_t first, size_t last);
    void flush(Conn *c);
    void close_conn(Conn *c);
    uint32_t gpu_of(std::string_view key) const {
        return (uint32_t)((pmc_key_hash(key.data(), key.size()) % shards) % gpus.size());
    }
    std::unordered_map<std::string, Entry> &shard_of(std::string_view key) {
        return index[pmc_key_hash(key.data(), key.size()) % shards];
    }
    size_t put_arena(const void *p, size_t n) {
        const size_t o = arena.size();
        arena.append((const char *)p, n);
        return o;
    }
};

void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK); }

int Server::run(int port) {
    signal(SIGPIPE, SIG_IGN);
    signal(SIGINT, on_signal);
    signal(SIGTERM, on_signal);
    index.resize(shards);
    lfd = socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    a.sin_port = htons((uint16_t)port);
    if (bind(lfd, (sockaddr *)&a, sizeof a) != 0 || listen(lfd, 1024) != 0) {
        perror("bind/listen");
        return 1;
    }
    set_nonblock(lfd);
    ep = epoll_create1(0);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = lfd;
    epoll_ctl(ep, EPOLL_CTL_ADD, lfd, &ev);
    printf("READY %d\n", port);
    fflush(stdout);
    std::vector<epoll_event> evs(2048);  // MAX_EVENTS (constants.hpp:7)
    std::vector<Conn *> ready;
    while (!g_stop) {
        const int k = epoll_wait(ep, evs.data(), (int)evs.size(), 100);  // EPOLL_WAIT_TIMEOUT_MSEC
        if (k < 0) {
            if (errno == EINTR) continue;
            perror("epoll_wait");
            break;
        }
        ready.clear();
        for (int i = 0; i < k; i++) {
            if (evs[i].data.fd == lfd) {
                accept_all();
                continue;
            }
            auto it = conns.find(evs[i].data.fd);
            if (it == conns.end()) continue;
            Conn *c = it->second.get();
            if (evs[i].events & EPOLLOUT) flush(c);
            if (evs[i].events & (EPOLLIN | EPOLLERR | EPOLLHUP)) {
                read_conn(c);
                ready.push_back(c);
            }
        }
        if (ready.empty()) continue;
        const double t_it = now_s();
        // one batch: every complete request of every ready connection
        reqs.clear();
        arena.clear();
        tx_keep.clear();
        for (auto &g : gpus) {
            g.puts.clear();
            g.gets.clear();
            g.get_frame.clear();
        }
        std::vector<std::pair<size_t, size_t>> span(ready.size());
        for (size_t j = 0; j < ready.size(); j++) {
            span[j].first = reqs.size();
            frame(ready[j]);
            span[j].second = reqs.size();
        }
        process();
        for (size_t j = 0; j < ready.size(); j++) send_conn(ready[j], span[j].first, span[j].second);
        for (Conn *c : ready) {
            c->in.erase(0, c->parsed);
            c->parsed = 0;
            if (c->closing && c->out.empty()) close_conn(c);
        }
        for (auto &g : gpus)  // replaced / deleted extents: their GETs have run
            if (!g.to_free.empty()) {
                pmc_store_free(g.store, g.to_free.data(), (uint32_t)g.to_free.size());
                g.to_free.clear();
            }
        st.iterations++;
        st.t_iter += now_s() - t_it;
    }
    printf("{\"iterations\": %llu, \"requests\": %llu, \"resp_requests\": %llu, \"sets\": %llu, \"gets\": %llu, \"dels\": %llu, "
           "\"compressed\": %llu, \"decompressed\": %llu, \"raw_fallbacks\": %llu, \"pending_hits\": %llu, "
           "\"put_calls\": %llu, \"get_calls\": %llu, \"t_iter\": %.4f, \"t_codec\": %.4f, \"t_put\": %.4f, "
           "\"t_get\": %.4f}\n",
           (unsigned long long)st.iterations, (unsigned long long)st.requests,
           (unsigned long long)st.resp_requests, (unsigned long long)st.sets,
           (unsigned long long)st.gets, (unsigned long long)st.dels, (unsigned long long)st.compressed,
           (unsigned long long)st.decompressed, (unsigned long long)st.raw_fallbacks,
           (unsigned long long)st.pending_hits, (unsigned long long)st.put_calls, (unsigned long long)st.get_calls,
           st.t_iter, st.t_codec, st.t_put, st.t_get);
    fflush(stdout);
    return 0;
}

void Server::accept_all() {
    for (;;) {
        int fd = accept(lfd, nullptr, nullptr);
        if (fd < 0) return;
        set_nonblock(fd);
        int one = 1;
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        auto c = std::make_unique<Conn>();
        c->fd = fd;
        epoll_event ev{};
        ev.events = EPOLLIN;
        ev.data.fd = fd;
        epoll_ctl(ep, EPOLL_CTL_ADD, fd, &ev);
        conns[fd] = std::move(c);
    }
}

void Server::read_conn(Conn *c) {
    char buf[16384];  // READ_BUFFER_SIZE (constants.hpp:9)
    for (;;) {
        const ssize_t r = read(c->fd, buf, sizeof buf);
        if (r > 0) {
            c->in.append(buf, (size_t)r);
            continue;
        }
        if (r == 0) c->closing = true;
        else if (errno == EINTR) continue;
        else if (errno != EAGAIN && errno != EWOULDBLOCK) c->closing = true;
        return;
    }
}

// RESP framing (parseRespMessageLength, protocol.cpp:294-356): "*<n>\r\n" then n bulk strings
// "$<len>\r\n<bytes>\r\n".  Returns the message length, 0 = incomplete, SIZE_MAX = malformed.
size_t resp_message_length(const char *b, size_t start, size_t end) {
    size_t idx = start + 1;
    auto number = [&](size_t &out) -> int {  // 1 ok, 0 incomplete, -1 error
        size_t v = 0;
        bool any = false;
        while (idx < end) {
            const char c = b[idx];
            if (c == '\r') {
                if (idx + 1 >= end || b[idx + 1] != '\n' || !any) return -1;  // (the reference: Error here)
                idx += 2;
                out = v;
                return 1;
            }
            if (c < '0' || c > '9') return -1;
            any = true;
            v = v * 10 + (size_t)(c - '0');
            idx++;
        }
        return any ? 0 : -1;  // (protocol.cpp:321: no digit before the end is an Error, digits are not)
    };
    size_t n = 0;
    int k = number(n);
    if (k <= 0) return k < 0 ? SIZE_MAX : 0;
    for (size_t a = 0; a < n; a++) {
        if (idx >= end) return 0;
        if (b[idx] != '$') return SIZE_MAX;
        idx++;
        size_t len = 0;
        k = number(len);
        if (k <= 0) return k < 0 ? SIZE_MAX : 0;
        if (idx + len + 2 > end) return 0;
        idx += len;
        if (b[idx] != '\r' || b[idx + 1] != '\n') return SIZE_MAX;
        idx += 2;
    }
    return idx - start;
}

// custom requests end at 0x1F, empty ones are skipped; a '*' starts a RESP array (readRequestAsync,
// server.cpp:433-479).  A malformed RESP array closes the connection and drops every request framed from
// this read (server.cpp:448-455): so the whole read is framed before any request is applied.
void Server::frame(Conn *c) {
    struct Span {
        size_t pos, len;
        uint8_t proto;
    };
    std::vector<Span> spans;
    size_t pos = c->parsed;
    const char *b = c->in.data();
    const size_t end = c->in.size();
    for (;;) {
        while (pos < end && b[pos] == kSep) pos++;
        if (pos >= end) break;
        if (b[pos] == '*') {
            const size_t n = resp_message_length(b, pos, end);
            if (n == 0) break;
            if (n == SIZE_MAX) {
                c->closing = true;
                c->parsed = end;
                return;
            }
            spans.push_back(Span{pos, n, kResp});
            pos += n;
            continue;
        }
        const size_t e = c->in.find(kSep, pos);
        if (e == std::string::npos) break;
        spans.push_back(Span{pos, e - pos, kCustom});
        pos = e + 1;
    }
    c->parsed = pos;
    for (const Span &sp : spans) {
        const std::string_view payload(b + sp.pos, sp.len);
        if (sp.proto == kResp) apply_resp(c, push_req(c, kResp), payload);
        else apply(push_req(c, kCustom), payload);
    }
}

// one custom request, in order, against the index (processRequestSync server.cpp:282-321)
void Server::apply(size_t q, std::string_view payload) {
    st.requests++;
    Resp &r = reqs[q].r;
    r.kind = kStatic;
    const size_t sp1 = payload.find(' ');
    if (sp1 == std::string_view::npos) {
        r.p = kUnparsable;
        return;
    }
    const std::string_view cmd = payload.substr(0, sp1), rest = payload.substr(sp1 + 1);
    if (rest.empty()) {
        r.p = kBadFormat;
        return;
    }
    const size_t sp2 = rest.find(' ');
    const std::string_view key = rest.substr(0, sp2);
    const bool has_val = sp2 != std::string_view::npos;
    if (cmd == "SET") {
        if (!has_val) {
            r.p = kBadFormat;
            return;
        }
        do_set(r, key, rest.substr(sp2 + 1));
        return;
    }
    if (cmd == "GET") return do_get(r, key);
    if (cmd == "DEL") return do_del(r, key);
    r.p = kUnknown;
}

// one RESP request (processRequestSync server.cpp:147-280; parseRespCommand protocol.cpp:358-397)
void Server::apply_resp(Conn *c, size_t q, std::string_view payload) {
    st.requests++;
    st.resp_requests++;
    reqs[q].r.kind = kStatic;
    auto fail = [&](const char *err) {  // ++numErrors; markRespTransactionError
        if (c->tx_active) c->tx_aborted = true;
        reqs[q].r.p = err;
    };
    // parts: 1-3 bulk strings; each is a C string to the reference (it writes a NUL at its CR)
    std::string_view part[3];
    size_t argc = 0, idx = 1;
    const char *b = payload.data();
    const size_t end = payload.size();
    auto number = [&](size_t &out) {
        size_t v = 0;
        bool any = false;
        while (idx < end && b[idx] >= '0' && b[idx] <= '9') v = v * 10 + (size_t)(b[idx++] - '0'), any = true;
        if (!any || idx + 1 >= end || b[idx] != '\r' || b[idx + 1] != '\n') return false;
        idx += 2;
        out = v;
        return true;
    };
    bool ok = number(argc) && argc >= 1 && argc <= 3;
    for (size_t i = 0; ok && i < argc; i++) {
        size_t len = 0;
        ok = idx < end && b[idx++] == '$' && number(len) && idx + len + 2 <= end;
        if (ok) {
            part[i] = std::string_view(b + idx, strnlen(b + idx, len));
            idx += len + 2;
        }
    }
    if (!ok) return fail(kRespErrUnparsable);
    const std::string_view cmd = part[0];
    Resp &r = reqs[q].r;
    if (cmd == "MULTI") {
        if (c->tx_active) return fail(kRespErrNested);
        c->tx_active = true;
        c->tx_aborted = false;
        c->tx.clear();
        r.p = kRespOK;
        return;
    }
    if (cmd == "DISCARD") {
        if (!c->tx_active) {
            r.p = kRespErrDiscardNoMulti;
            return;
        }
        c->tx.clear();
        c->tx_active = c->tx_aborted = false;
        r.p = kRespOK;
        return;
    }
    if (cmd == "EXEC") {
        if (!c->tx_active) {
            r.p = kRespErrExecNoMulti;
            return;
        }
        const bool aborted = c->tx_aborted;
        c->tx_active = c->tx_aborted = false;
        if (aborted) {
            c->tx.clear();
            r.p = kRespErrExecAborted;
            return;
        }
        // makeRespArray (protocol.cpp:499-533): "*<n>\r\n" and the n replies, each its own Resp here
        tx_keep.push_back(std::move(c->tx));
        c->tx.clear();
        const std::vector<TxCmd> &queue = tx_keep.back();
        char hdr[32];
        const int hn = snprintf(hdr, sizeof hdr, "*%zu\r\n", queue.size());
        r.kind = kArena;
        r.n = (size_t)hn;
        r.off = put_arena(hdr, r.n);
        for (const TxCmd &t : queue) {
            const size_t e = push_req(c, kResp);
            Resp &er = reqs[e].r;
            er.kind = kStatic;
            if (t.type == kGet) do_get(er, t.key);
            else if (t.type == kSet) do_set(er, t.key, t.val);
            else do_del(er, t.key);
        }
        return;
    }
    const uint8_t type = cmd == "GET" ? kGet : cmd == "SET" ? kSet : cmd == "DEL" ? kDel : 0xFF;
    if (type == 0xFF) return fail(kRespErrUnknown);
    if (argc != (type == kSet ? 3u : 2u)) return fail(kRespErrBadFormat);
    if (c->tx_active) {  // queueRespCommand
        c->tx.push_back(TxCmd{type, std::string(part[1]), std::string(type == kSet ? part[2] : std::string_view())});
        r.p = kRespQueued;
        return;
    }
    if (type == kGet) do_get(r, part[1]);
    else if (type == kSet) do_set(r, part[1], part[2]);
    else do_del(r, part[1]);
}

// "$<len>\r\n" value "\r\n" into the arena (makeRespBulkString, protocol.cpp:466-497)
void Server::resp_bulk_arena(Resp &r, const char *p, size_t n) {
    char hdr[32];
    const int hn = snprintf(hdr, sizeof hdr, "$%zu\r\n", n);
    r.kind = kArena;
    r.off = put_arena(hdr, (size_t)hn);
    put_arena(p, n);
    put_arena("\r\n", 2);
    r.n = (size_t)hn + n + 2;
}

// SET / GET / DEL against the index (KeyValueStore semantics, kvs.cpp:141-235); r.proto picks the reply
void Server::do_set(Resp &r, std::string_view key, std::string_view val) {
    st.sets++;
    val = val.substr(0, strnlen(val.data(), val.size()));  // a C string (kvs.cpp:148 strlen)
    const uint32_t g = gpu_of(key);
    Entry &e = shard_of(key)[std::string(key)];
    if (e.kind == kDevice) gpus[e.gpu].to_free.push_back(e.ext);
    e.gpu = g;
    if (codec != Codec::kOff && val.size() + 1 >= kMinCompress) {
        if (codec == Codec::kBatch) {
            e.kind = kPending;
            std::string().swap(e.bytes);  // an earlier raw / host-gzip value leaves host memory
            e.put = (uint32_t)gpus[g].puts.size();
            gpus[g].puts.push_back(Put{key, val});
        } else {  // single-value call, as the unchanged server through the drop-in
            e.bytes.resize(pmc_gzip_bound(val.size()));
            size_t n = 0;
            if (pmc_gzip_compress(gpus[g].ctx, val.data(), val.size(), e.bytes.data(), e.bytes.size(), &n) == 0) {
                e.bytes.resize(n);
                e.kind = kHostGz;
                st.compressed++;
            } else {
                e.bytes.assign(val.data(), val.size());
                e.kind = kRaw;
                st.raw_fallbacks++;
            }
        }
    } else {
        e.kind = kRaw;
        e.bytes.assign(val.data(), val.size());
    }
    r.p = r.proto == kResp ? kRespOK : kOK;
}

void Server::do_get(Resp &r, std::string_view key) {
    st.gets++;
    const bool resp = r.proto == kResp;
    auto &m = shard_of(key);
    auto it = m.find(std::string(key));
    if (it == m.end()) {
        r.p = resp ? kRespNil : kNil;
        return;
    }
    Entry &e = it->second;
    if (e.kind == kRaw) {  // copied: a later SET in this iteration may replace it
        if (resp) return resp_bulk_arena(r, e.bytes.data(), e.bytes.size());
        r.kind = kArena;
        r.n = e.bytes.size();
        r.off = put_arena(e.bytes.data(), r.n);
    } else if (e.kind == kPending) {  // SET earlier in this iteration: its own bytes
        const Put &pt = gpus[e.gpu].puts[e.put];
        st.pending_hits++;
        if (resp) return resp_bulk_arena(r, pt.val.data(), pt.val.size());
        r.kind = kView;
        r.p = pt.val.data();
        r.n = pt.val.size();
    } else if (e.kind == kDevice) {
        r.kind = kStoreGet;
        r.gpu = e.gpu;
        r.off = gpus[e.gpu].gets.size();
        gpus[e.gpu].gets.push_back(e.ext);
        gpus[e.gpu].get_frame.push_back(resp ? PMC_FRAME_RESP : PMC_FRAME_CUSTOM);
    } else {  // kHostGz: single-value decompress now
        const uint32_t cap = pmc_gzip_isize(e.bytes.data(), e.bytes.size());
        std::string v(cap + 1, '\0');
        size_t n = 0;
        if (pmc_gzip_decompress(gpus[e.gpu].ctx, e.bytes.data(), e.bytes.size(), v.data(), cap + 1, &n) == 0) {
            st.decompressed++;
            if (resp) return resp_bulk_arena(r, v.data(), n);
            r.kind = kArena;
            r.n = n;
            r.off = put_arena(v.data(), n);
        } else {
            r.p = resp ? kRespNil : kNil;  // decompressEntry's nullptr (kvs.cpp:234) -> NOTHING (shard.cpp:30)
        }
    }
}

void Server::do_del(Resp &r, std::string_view key) {
    st.dels++;
    const bool resp = r.proto == kResp;
    auto &m = shard_of(key);
    auto it = m.find(std::string(key));
    if (it == m.end()) {  // KEY_NOT_EXISTS; RESP: integer 0 (server.cpp:135-142)
        r.p = resp ? kRespZero : kKeyNotExists;
        return;
    }
    if (it->second.kind == kDevice) gpus[it->second.gpu].to_free.push_back(it->second.ext);
    m.erase(it);  // a pending put of this key is released once it ran (run_codec)
    r.p = resp ? kRespOne : kOK;
}

void Server::process() {
    if (codec != Codec::kBatch) return;
    const double t0 = now_s();
    run_codec();
    st.t_codec += now_s() - t0;
}

// the iteration's codec work: one put batch and one get batch per GPU; the put (compress stream)
// and the get (decompress stream) of a GPU run side by side, and GPUs on their own threads
void Server::run_codec() {
    auto work = [&](Gpu &g) {
        g.err = 0;
        int gerr = 0;
        const uint32_t np = (uint32_t)g.puts.size(), ng = (uint32_t)g.gets.size();
        std::thread getter;
        if (ng) {
            g.get_resp.assign(ng, nullptr);
            g.get_len.assign(ng, 0);
            g.get_rc.assign(ng, 0);
            getter = std::thread([&] {
                const double t0 = now_s();
                gerr = pmc_store_get_batch_frames(g.store, g.gets.data(), ng, g.get_frame.data(), g.get_resp.data(),
                                                  g.get_len.data(), g.get_rc.data());
                if (&g == &gpus[0]) {
                    st.t_get += now_s() - t0;
                    st.get_calls++;
                }
            });
        }
        if (np) {
            std::string blob;
            std::vector<uint64_t> off(np);
            std::vector<uint32_t> len(np);
            for (uint32_t j = 0; j < np; j++) {
                off[j] = blob.size();
                len[j] = (uint32_t)g.puts[j].val.size();
                blob.append(g.puts[j].val);
            }
            g.put_ext.assign(np, pmc_extent{});
            g.put_rc.assign(np, 0);
            const double t0 = now_s();
            g.err = pmc_store_put_batch(g.store, (const uint8_t *)blob.data(), off.data(), len.data(), np,
                                        g.put_ext.data(), g.put_rc.data());
            if (&g == &gpus[0]) {
                st.t_put += now_s() - t0;
                st.put_calls++;
            }
        }
        if (getter.joinable()) getter.join();
        if (gerr) g.err = gerr;
    };
    if (gpus.size() == 1) {
        work(gpus[0]);
    } else {
        std::vector<std::thread> th;
        for (size_t k = 1; k < gpus.size(); k++) th.emplace_back([&, k] { work(gpus[k]); });
        work(gpus[0]);
        for (auto &t : th) t.join();
    }
    // commit the puts: the entry still waiting for put j gets its extent; a failed compression
    // stores the raw value (kvs.cpp:188-192); a put superseded or deleted in the iteration is released
    for (uint32_t k = 0; k < gpus.size(); k++) {
        Gpu &g = gpus[k];
        for (uint32_t j = 0; j < g.puts.size(); j++) {
            const bool ok = !g.err && g.put_rc[j] == 0;
            auto &m = shard_of(g.puts[j].key);
            auto it = m.find(std::string(g.puts[j].key));
            const bool live = it != m.end() && it->second.kind == kPending && it->second.gpu == k && it->second.put == j;
            if (!live) {
                if (ok) g.to_free.push_back(g.put_ext[j]);
                continue;
            }
            if (ok) {
                it->second.kind = kDevice;
                it->second.ext = g.put_ext[j];
                std::string().swap(it->second.bytes);
                st.compressed++;
            } else {
                it->second.kind = kRaw;
                it->second.bytes.assign(g.puts[j].val.data(), g.puts[j].val.size());
                st.raw_fallbacks++;
            }
        }
        st.decompressed += g.gets.size();
    }
}

void Server::send_conn(Conn *c, size_t first, size_t last) {
    std::vector<iovec> iov;
    iov.reserve((last - first) * 2);
    static const char sep = kSep;
    for (size_t i = first; i < last; i++) {
        const Resp &r = reqs[i].r;
        const bool custom = r.proto == kCustom;  // RESP replies carry their own framing (server.cpp:555)
        switch (r.kind) {
        case kStatic:
            iov.push_back({(void *)r.p, strlen(r.p)});
            break;
        case kArena:
            iov.push_back({(void *)(arena.data() + r.off), r.n});
            break;
        case kView:
            iov.push_back({(void *)r.p, r.n});
            break;
        case kStoreGet: {
            Gpu &g = gpus[r.gpu];
            if (g.err || g.get_rc[r.off] != 0) {  // decompressEntry -> nullptr -> "(nil)" / "$-1\r\n"
                iov.push_back({(void *)(custom ? kNil : kRespNil), custom ? sizeof kNil - 1 : sizeof kRespNil - 1});
            } else {  // value + 0x1F, or "$<len>\r\n" value "\r\n", framed in the pinned image
                iov.push_back({(void *)g.get_resp[r.off], g.get_len[r.off]});
                continue;
            }
            break;
        }
        }
        if (custom) iov.push_back({(void *)&sep, 1});
    }
    size_t k = 0;
    if (c->out.empty()) {
        while (k < iov.size()) {
            msghdr msg{};
            msg.msg_iov = &iov[k];
            msg.msg_iovlen = std::min<size_t>(iov.size() - k, 1024);
            const ssize_t s = sendmsg(c->fd, &msg, MSG_NOSIGNAL);
            if (s < 0) {
                if (errno == EINTR) continue;
                if (errno != EAGAIN && errno != EWOULDBLOCK) {
                    c->closing = true;
                    return;
                }
                break;
            }
            size_t left = (size_t)s;
            while (left && k < iov.size()) {
                if (left >= iov[k].iov_len) {
                    left -= iov[k].iov_len;
                    k++;
                } else {
                    iov[k].iov_base = (char *)iov[k].iov_base + left;
                    iov[k].iov_len -= left;
                    left = 0;
                }
            }
        }
    }
    if (k < iov.size()) {  // the socket is full: keep the rest (the pinned image is reused next batch)
        for (; k < iov.size(); k++) c->out.append((const char *)iov[k].iov_base, iov[k].iov_len);
        epoll_event ev{};
        ev.events = EPOLLIN | EPOLLOUT;
        ev.data.fd = c->fd;
        epoll_ctl(ep, EPOLL_CTL_MOD, c->fd, &ev);
    }
}

void Server::flush(Conn *c) {
    while (!c->out.empty()) {
        const ssize_t s = send(c->fd, c->out.data(), c->out.size(), MSG_NOSIGNAL);
        if (s < 0) {
            if (errno == EINTR) continue;
            if (errno != EAGAIN && errno != EWOULDBLOCK) c->closing = true;
            return;
        }
        c->out.erase(0, (size_t)s);
    }
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = c->fd;
    epoll_ctl(ep, EPOLL_CTL_MOD, c->fd, &ev);
}

void Server::close_conn(Conn *c) {
    epoll_ctl(ep, EPOLL_CTL_DEL, c->fd, nullptr);
    close(c->fd);
    conns.erase(c->fd);
}

} // namespace

int main(int argc, char **argv) {
    int port = 9001, ngpu = 1;
    uint64_t heap_mb = 4096;
    Server s;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string a = argv[i], v = argv[i + 1];
        if (a == "--port") port = atoi(v.c_str());
        else if (a == "--gpus") ngpu = atoi(v.c_str());
        else if (a == "--shards") s.shards = (uint32_t)atoi(v.c_str());
        else if (a == "--heap-mb") heap_mb = strtoull(v.c_str(), nullptr, 10);
        else if (a == "--codec") s.codec = v == "single" ? Codec::kSingle : v == "off" ? Codec::kOff : Codec::kBatch;
        else {
            fprintf(stderr, "unknown option %s\n", a.c_str());
            return 2;
        }
    }
    if (ngpu < 1 || s.shards < 1) return 2;
    s.gpus.resize(ngpu);
    for (int k = 0; k < ngpu; k++) {
        if (s.codec == Codec::kOff) break;
        if (pmc_ctx_create(k, &s.gpus[k].ctx) != PMC_OK) {
            fprintf(stderr, "pmc_ctx_create(%d): %s\n", k, pmc_last_error());
            return 1;
        }
        if (s.codec == Codec::kBatch && pmc_store_create(s.gpus[k].ctx, heap_mb << 20, &s.gpus[k].store) != PMC_OK) {
            fprintf(stderr, "pmc_store_create(%d): %s\n", k, pmc_last_error());
            return 1;
        }
    }
    const int rc = s.run(port);
    for (auto &g : s.gpus) {
        if (g.store) pmc_store_destroy(g.store);
        if (g.ctx) pmc_ctx_destroy(g.ctx);
    }
    return rc;
}
