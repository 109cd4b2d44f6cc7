// pmc_loadgen.cpp -- pipelined custom-protocol load against pmc_server (or any server speaking it).
//
// Shaped like the reference's load test in pipeline mode (/root/reference/tests/tcp_server_test.py
// :158-244, `-p -b 100`): each connection writes batches of B commands joined by 0x1F and then reads
// B responses; connections run on their own threads.  Unlike that test, whose values (`value{i}`,
// <= 12 chars) never reach the codec, values here are JSON slices of the reference's
// tests/data corpus (SURVEY §8d generator), so every SET compresses and every GET decompresses.
//
// usage: pmc_loadgen --port P --data DIR [--conns 16] [--keys 65536] [--vlen 4096] [--batch 100]
//                    [--ops 200000] [--mix 50]       (percent of SETs in the timed phase)
//                    [--proto custom|resp]           (resp: commands as RESP arrays, as the reference's
//                                                     tcp_server_test.py --resp sends them through redis-py)
// Phases: preload (SET every key once, untimed), then --ops timed commands over random keys,
// every GET checked against the last value SET for its key.  Prints one JSON line.
#include <arpa/inet.h>
#include <dirent.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace {

uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Opts {
    int port = 9001, conns = 16, batch = 100, mix = 50, warmup_sec = 60;
    uint64_t keys = 65536, vlen = 4096, ops = 200000;
    std::string data;
    bool resp = false;
};
bool g_resp = false;

std::string corpus;

// value of key k at version v: a corpus slice (splitmix64(seed ^ i) % (len - V + 1))
std::string value_of(uint64_t k, uint64_t v, uint64_t vlen) {
    const uint64_t off = splitmix64(0x5EEDull ^ (k * 1000003ull + v)) % (corpus.size() - vlen + 1);
    return corpus.substr(off, vlen);
}

int connect_to(int port) {
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (connect(fd, (sockaddr *)&a, sizeof a) != 0) {
        close(fd);
        return -1;
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    return fd;
}

// Writes the batch and reads its n responses (0x1F-terminated) into out, reading while it writes: a
// server that answers the first requests of a batch before it has read the last ones (the reference
// server sends each epoll iteration's responses before reading again, server.cpp:386-390, and spins on
// EAGAIN until they are sent) would otherwise deadlock against a client still blocked in send().
// One reply at pos: custom replies end at 0x1F (kept out of the reply), RESP replies are a "+ - :" line or a
// "$<len>\r\n" bulk string (kept whole).  Returns the reply's end (npos: incomplete); *next: past it.
size_t reply_end(const std::string &b, size_t pos, size_t *next) {
    if (!g_resp) {
        const size_t e = b.find('\x1f', pos);
        if (e != std::string::npos) *next = e + 1;
        return e;
    }
    const size_t e = b.find("\r\n", pos);
    if (e == std::string::npos) return e;
    if (b[pos] != '$' || b[pos + 1] == '-') return *next = e + 2;
    const size_t end = e + 2 + strtoull(b.c_str() + pos + 1, nullptr, 10) + 2;
    if (b.size() < end) return std::string::npos;
    return *next = end;
}

std::string bulk(const std::string &v) { return "$" + std::to_string(v.size()) + "\r\n" + v + "\r\n"; }
std::string resp_cmd(std::initializer_list<const std::string *> parts) {
    std::string r = "*" + std::to_string(parts.size()) + "\r\n";
    for (const std::string *p : parts) r += bulk(*p);
    return r;
}

bool exchange(int fd, const std::string &req, std::string &buf, size_t n, std::vector<std::string> &out) {
    out.clear();
    size_t sent = 0, pos = 0;
    char tmp[1 << 16];
    while (out.size() < n) {
        size_t next = 0;
        const size_t e = pos < buf.size() ? reply_end(buf, pos, &next) : std::string::npos;
        if (e != std::string::npos) {
            out.emplace_back(buf, pos, e - pos);
            pos = next;
            continue;
        }
        buf.erase(0, pos);
        pos = 0;
        pollfd pf{fd, (short)(POLLIN | (sent < req.size() ? POLLOUT : 0)), 0};
        if (poll(&pf, 1, 60000) <= 0) return false;
        if (pf.revents & (POLLERR | POLLHUP | POLLNVAL)) return false;
        if ((pf.revents & POLLOUT) && sent < req.size()) {
            const ssize_t w = send(fd, req.data() + sent, req.size() - sent, MSG_NOSIGNAL | MSG_DONTWAIT);
            if (w < 0 && errno != EAGAIN && errno != EWOULDBLOCK) return false;
            if (w > 0) sent += (size_t)w;
        }
        if (pf.revents & POLLIN) {
            const ssize_t r = recv(fd, tmp, sizeof tmp, MSG_DONTWAIT);
            if (r == 0) return false;
            if (r < 0 && errno != EAGAIN && errno != EWOULDBLOCK) return false;
            if (r > 0) buf.append(tmp, (size_t)r);
        }
    }
    buf.erase(0, pos);
    return sent == req.size();
}

// Until the server answers a throwaway GET (up to `secs`): the reference CacheServer listens ~2 s before
// it accepts (its constructor sieves primes for every shard), and a request waiting in the backlog is
// read the moment its fd joins the epoll set, inside the connect race of
// /root/reference/src/server/conn_manager.hpp:83-93 (epoll registration before the ConnectionData is
// recorded) and server.cpp:373,409 (that map read without its lock), where it may never be answered.
// A reference server whose accept thread has self-deadlocked (validateConnections holds conn_mutex and
// calls closeConnection, which locks it again: conn_manager.hpp:109, :117, :142) never answers; the
// caller restarts it (scripts/ref_server_bench.sh), so a short --warmup-sec keeps that cheap.
bool warm_up(int port, int secs) {
    const auto t0 = std::chrono::steady_clock::now();
    std::string buf;
    std::vector<std::string> out;
    while (std::chrono::steady_clock::now() - t0 < std::chrono::seconds(secs)) {
        const int fd = connect_to(port);
        if (fd >= 0) {
            pollfd pf{fd, POLLOUT, 0};
            static const std::string wk = "__warmup__", get = "GET";
            const std::string req = g_resp ? resp_cmd({&get, &wk}) : "GET __warmup__\x1f";
            bool ok = send(fd, req.data(), req.size(), MSG_NOSIGNAL) == (ssize_t)req.size();
            pf.events = POLLIN;
            ok = ok && poll(&pf, 1, 1000) > 0 && (pf.revents & POLLIN);
            char tmp[256];
            ok = ok && recv(fd, tmp, sizeof tmp, 0) > 0;
            close(fd);
            if (ok) return true;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
    return false;
}

struct Worker {
    uint64_t ops = 0, sets = 0, gets = 0, bytes = 0, bad = 0;
};

} // namespace

int main(int argc, char **argv) {
    Opts o;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string a = argv[i], v = argv[i + 1];
        if (a == "--port") o.port = atoi(v.c_str());
        else if (a == "--conns") o.conns = atoi(v.c_str());
        else if (a == "--keys") o.keys = strtoull(v.c_str(), nullptr, 10);
        else if (a == "--vlen") o.vlen = strtoull(v.c_str(), nullptr, 10);
        else if (a == "--batch") o.batch = atoi(v.c_str());
        else if (a == "--ops") o.ops = strtoull(v.c_str(), nullptr, 10);
        else if (a == "--mix") o.mix = atoi(v.c_str());
        else if (a == "--data") o.data = v;
        else if (a == "--warmup-sec") o.warmup_sec = atoi(v.c_str());
        else if (a == "--proto") o.resp = g_resp = v == "resp";
        else {
            fprintf(stderr, "unknown option %s\n", a.c_str());
            return 2;
        }
    }
    std::vector<std::string> names;
    if (DIR *d = opendir(o.data.c_str())) {
        while (dirent *e = readdir(d)) {
            std::string n = e->d_name;
            if (n.size() > 5 && n.substr(n.size() - 5) == ".json") names.push_back(n);
        }
        closedir(d);
    }
    std::sort(names.begin(), names.end());
    for (auto &n : names) {
        std::ifstream f(o.data + "/" + n, std::ios::binary);
        std::stringstream ss;
        ss << f.rdbuf();
        corpus += ss.str();
    }
    if (corpus.size() < o.vlen + 1) {
        fprintf(stderr, "corpus too small (%zu B from %s)\n", corpus.size(), o.data.c_str());
        return 2;
    }
    // keys are owned by connections (key % conns), so each connection knows its keys' versions
    std::vector<Worker> w(o.conns);
    std::atomic<int> failed{0};
    auto run_phase = [&](bool preload) {
        std::vector<std::thread> th;
        for (int c = 0; c < o.conns; c++)
            th.emplace_back([&, c] {
                const int fd = connect_to(o.port);
                if (fd < 0) {
                    failed++;
                    return;
                }
                // (the first write 20 ms after the connect, past the reference server's registration window)
                std::this_thread::sleep_for(std::chrono::milliseconds(20));
                std::vector<uint64_t> mine;
                for (uint64_t k = c; k < o.keys; k += o.conns) mine.push_back(k);
                std::vector<uint64_t> ver(mine.size(), 0);
                if (!preload) {  // versions after the preload
                    for (auto &v : ver) v = 1;
                }
                uint64_t rng = splitmix64(0x7ull + c), todo = preload ? mine.size() : o.ops / o.conns, done = 0;
                std::string buf, req;
                std::vector<std::string> resp;
                std::vector<std::pair<int, std::string>> expect;  // 0 = SET (OK), 1 = GET (value)
                Worker &me = w[c];
                while (done < todo) {
                    req.clear();
                    expect.clear();
                    const uint64_t b = std::min<uint64_t>(o.batch, todo - done);
                    for (uint64_t j = 0; j < b; j++) {
                        size_t ki;
                        bool set;
                        if (preload) {
                            ki = done + j;
                            set = true;
                        } else {
                            rng = splitmix64(rng);
                            ki = rng % mine.size();
                            set = (int)((rng >> 40) % 100) < o.mix;
                        }
                        const uint64_t k = mine[ki];
                        static const std::string kSet = "SET", kGet = "GET";
                        const std::string key = "key" + std::to_string(k);
                        if (set) {
                            const std::string v = value_of(k, ++ver[ki], o.vlen);
                            req += o.resp ? resp_cmd({&kSet, &key, &v}) : "SET " + key + " " + v + '\x1f';
                            expect.emplace_back(0, o.resp ? "+OK\r\n" : "OK");
                            me.sets++;
                        } else {
                            req += o.resp ? resp_cmd({&kGet, &key}) : "GET " + key + '\x1f';
                            const std::string v = value_of(k, ver[ki], o.vlen);
                            expect.emplace_back(1, o.resp ? bulk(v) : v);
                            me.gets++;
                        }
                        me.bytes += o.vlen;
                    }
                    if (!exchange(fd, req, buf, b, resp)) {
                        failed++;
                        break;
                    }
                    for (uint64_t j = 0; j < b; j++)
                        if (resp[j] != expect[j].second) me.bad++;
                    done += b;
                    me.ops += b;
                }
                close(fd);
            });
        for (auto &t : th) t.join();
    };
    if (!warm_up(o.port, o.warmup_sec)) {
        fprintf(stderr, "server on port %d did not answer within %d s\n", o.port, o.warmup_sec);
        return 1;
    }
    run_phase(true);
    for (auto &x : w) x = Worker{};
    const auto t0 = std::chrono::steady_clock::now();
    run_phase(false);
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    Worker s;
    for (auto &x : w) {
        s.ops += x.ops;
        s.sets += x.sets;
        s.gets += x.gets;
        s.bytes += x.bytes;
        s.bad += x.bad;
    }
    printf("{\"ops\": %llu, \"sets\": %llu, \"gets\": %llu, \"seconds\": %.4f, \"ops_per_s\": %.1f, "
           "\"value_gib_s\": %.4f, \"mismatches\": %llu, \"failed_conns\": %d, \"conns\": %d, \"batch\": %d, "
           "\"vlen\": %llu, \"keys\": %llu, \"set_pct\": %d, \"proto\": \"%s\"}\n",
           (unsigned long long)s.ops, (unsigned long long)s.sets, (unsigned long long)s.gets, t, s.ops / t,
           s.bytes / t / (1ull << 30), (unsigned long long)s.bad, failed.load(), o.conns, o.batch,
           (unsigned long long)o.vlen, (unsigned long long)o.keys, o.mix, o.resp ? "resp" : "custom");
    return (s.bad || failed) ? 1 : 0;
}
