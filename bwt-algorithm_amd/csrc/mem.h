// mem.h -- large host blocks for the per-step arrays of the host stages.
//
// A 100 Mbp step touches ~1 GB of fresh host arrays (downloaded hits, fold
// items, speculative fold output, records, rendered rows).  Served by malloc,
// each step faults all of it in again 4 KiB at a time (measured: ~130-200k
// minor faults per post-processing call, a large share of its wall time).
// Blocks of >= kBigMin bytes therefore come from 2 MiB-aligned anonymous
// mappings advised for transparent huge pages, and freed blocks stay in a
// process-wide cache: the next step's arrays of the same sizes reuse
// already-faulted memory.
#pragma once

#include <cstddef>
#include <functional>
#include <new>
#include <utility>

namespace bwtmi {

constexpr size_t kBigMin = size_t(1) << 20;

void *big_alloc(size_t bytes);             // throws std::bad_alloc
void big_free(void *p, size_t bytes) noexcept;
size_t big_cached_bytes();                 // bytes held in the cache (tests / stats)
void big_trim();                           // unmap every cached block
// mapped size of the live block that starts at p (0 if p is not a block start)
size_t big_block_size(const void *p);
// called (under the cache lock) before a block is unmapped; the device layer
// uses it to drop its DMA registration of blocks it pinned (api.cpp)
void big_set_unmap_hook(void (*hook)(void *p, size_t bytes));

// Runs fn on a background thread, in submission order: releasing a step's
// large record sets overlaps the next step's device phase instead of
// delaying it.  defer_drain() waits for everything submitted so far.
void defer(std::function<void()> fn);
void defer_drain();

// While a DeferConstruct is alive on this thread, BigAlloc's no-argument
// construct() does nothing: a vector resized under it holds raw storage that
// the caller default-constructs itself, in parallel (a serial resize of 321k
// records spent ~5 ms of the C3 step), before any other use.
inline bool &big_defer_construct() {
    thread_local bool on = false;
    return on;
}
struct DeferConstruct {
    DeferConstruct() { big_defer_construct() = true; }
    ~DeferConstruct() { big_defer_construct() = false; }
    DeferConstruct(const DeferConstruct &) = delete;
    DeferConstruct &operator=(const DeferConstruct &) = delete;
};

// Allocator for vectors of trivially-copyable (or default-constructible)
// elements: small arrays from operator new, large ones from big_alloc.
// construct() without arguments default-initialises (no zero fill): arrays
// that are written once in parallel skip a serial value-initialisation pass.
template <class T>
struct BigAlloc {
    using value_type = T;
    BigAlloc() = default;
    template <class U>
    BigAlloc(const BigAlloc<U> &) noexcept {}
    template <class U>
    struct rebind {
        using other = BigAlloc<U>;
    };
    T *allocate(size_t n) {
        const size_t b = n * sizeof(T);
        if (b < kBigMin) return static_cast<T *>(::operator new(b));
        return static_cast<T *>(big_alloc(b));
    }
    void deallocate(T *p, size_t n) noexcept {
        const size_t b = n * sizeof(T);
        if (b < kBigMin) ::operator delete(p);
        else big_free(p, b);
    }
    template <class U>
    void construct(U *p) noexcept(noexcept(::new ((void *)p) U)) {
        if (!big_defer_construct()) ::new ((void *)p) U;
    }
    template <class U, class... A>
    void construct(U *p, A &&...a) {
        ::new ((void *)p) U(std::forward<A>(a)...);
    }
    template <class U>
    bool operator==(const BigAlloc<U> &) const noexcept { return true; }
    template <class U>
    bool operator!=(const BigAlloc<U> &) const noexcept { return false; }
};

}  // namespace bwtmi
