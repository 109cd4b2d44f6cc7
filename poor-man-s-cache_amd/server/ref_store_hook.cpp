// ref_store_hook.cpp -- SURVEY.md §8 f2 inside the reference's own KeyValueStore, unmodified.
//
// Linked into oracle/_ref/ref_server_store: the ref_server_batch build (the reference's server, kvs, hash and
// primegen sources compiled where they lie, ref_server_batch.patch, ref_batch_hook.cpp) plus this file, which
//   * puts the drop-in in device-store mode before main (pmc_batch::EnableDeviceStore): a compressed value's
//     Entry.value (/root/reference/src/kvs/kvs.hpp:38-44, set at kvs.cpp:185-187) is a 32-byte handle naming
//     the member's extent in HBM, not the member, so GET batches need no H2D of compressed bytes and the host
//     keeps no >= 16 KiB member buffer per value;
//   * replaces operator delete[]: MemoryPool::deallocate frees Entry.value with delete[] (kvs.hpp:87-98, on
//     SET over an existing key, DEL and resize), and a handle is recognised by its address (a slab of its
//     own) and releases its extent; every other pointer goes to free() as the default operator would.
// PMC_STORE_HEAP_MB sizes the device heap (default 16384).
#include <cstdlib>
#include <new>

#include "batch_codec.hpp"

namespace {
struct EnableStore {
    EnableStore() {
        const char *e = std::getenv("PMC_STORE_HEAP_MB");
        const unsigned long long mb = e ? std::strtoull(e, nullptr, 10) : 16384ull;
        pmc_batch::EnableDeviceStore((mb ? mb : 16384ull) << 20);
    }
} g_enable_store;
}  // namespace

void operator delete[](void *p) noexcept {
    if (p && pmc_batch::detail::ReleaseIfHandle(p)) return;
    std::free(p);
}
void operator delete[](void *p, std::size_t) noexcept { operator delete[](p); }
void operator delete[](void *p, const std::nothrow_t &) noexcept { operator delete[](p); }
