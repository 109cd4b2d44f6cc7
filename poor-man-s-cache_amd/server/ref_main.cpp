// ref_main.cpp -- a main() for the reference's own CacheServer without the Prometheus exposer.
//
// /root/reference/src/main.cpp:10-61 builds ServerSettings from the environment, starts a
// metrics::MetricsServer (prometheus-cpp, not in this image) and runs CacheServer::Start.  This main
// keeps everything but the exposer: the same variables and defaults (main.cpp:17-22), the same
// SIGINT/SIGTERM -> Stop() handling (:28-43), and a thread that drains the MetricsChannel the server
// pushes to (:45-58) so it does not grow.  The server itself is the reference's code, compiled where
// it lies (oracle/Makefile `server`); only the codec underneath kvs differs per binary:
//   ref_server_zlib   the reference's gzip_compressor.cpp + system zlib (the CPU baseline)
//   ref_server_dropin the drop-in GzipCompressor (libgzip_dropin.so, one GPU call per value)
//   ref_server_batch  the drop-in + ref_server_batch.patch + ref_batch_hook.cpp (one GPU batch per
//                     epoll iteration)
#include <atomic>
#include <chrono>
#include <csignal>
#include <functional>
#include <iostream>
#include <thread>

#include "env.hpp"
#include "server/server.hpp"

using namespace server;

namespace {
std::function<void(int)> g_on_signal;
void dispatch(int sig) {
    if (g_on_signal) g_on_signal(sig);
}
}  // namespace

int main() {
    MetricsChannel channel;
    const auto port = getFromEnv<int>("SERVER_PORT", true);
    const auto numShards = getFromEnv<uint_fast32_t>("NUM_SHARDS", false, 24);
    const auto sockBufferSize = getFromEnv<int>("SOCK_BUF_SIZE", false, 1048576);
    const auto connQueueLimit = getFromEnv<uint_fast32_t>("CONN_QUEUE_LIMIT", false, 1048576);
    const auto enableCompression = getFromEnv<bool>("ENABLE_COMPRESSION", false, true);
    const auto respInlineCapacity = getFromEnv<std::size_t>("RESP_INLINE_CAPACITY", false, static_cast<std::size_t>(255));
    ServerSettings settings{port, numShards, sockBufferSize, connQueueLimit, enableCompression, respInlineCapacity};
    CacheServer cacheServer{settings};
    g_on_signal = [&cacheServer](int sig) {
        if (sig == SIGINT || sig == SIGTERM) cacheServer.Stop();
    };
    std::signal(SIGINT, dispatch);
    std::signal(SIGTERM, dispatch);
    std::jthread drain([&channel](std::stop_token stop) {
        while (!stop.stop_requested()) {
            CacheServerMetrics m{0, 0, 0};
            while (channel.try_pop(m)) {
            }
            std::this_thread::sleep_for(std::chrono::milliseconds(200));
        }
    });
    return cacheServer.Start(channel);
}
