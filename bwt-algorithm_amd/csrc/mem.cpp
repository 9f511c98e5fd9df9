// mem.cpp -- cached, huge-page-advised host blocks (see mem.h).
#include "mem.h"

#include <sys/mman.h>

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <mutex>
#include <thread>
#include <unordered_map>

namespace bwtmi {
namespace {

constexpr size_t kHuge = size_t(2) << 20;
constexpr size_t kCacheCap = size_t(8) << 30;   // per process; one rank per GPU

struct Cache {
    std::mutex mu;
    std::multimap<size_t, void *> free_;        // mapped size -> cached block
    std::unordered_map<void *, size_t> live;    // block -> mapped size
    size_t cached = 0;
};

Cache &cache() {
    static Cache *c = new Cache;   // never destroyed: blocks may be freed during exit
    return *c;
}

void (*g_unmap_hook)(void *, size_t) = nullptr;

void unmap_block(void *p, size_t size) {
    if (g_unmap_hook) g_unmap_hook(p, size);
    munmap(p, size);
}

void *map_block(size_t size) {
    // over-map by 2 MiB and trim to a 2 MiB-aligned block so that every huge
    // page of it can be backed by a transparent huge page
    void *raw = mmap(nullptr, size + kHuge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (raw == MAP_FAILED) throw std::bad_alloc();
    const uintptr_t r = (uintptr_t)raw, a = (r + kHuge - 1) & ~(uintptr_t)(kHuge - 1);
    if (a > r) munmap(raw, a - r);
    const uintptr_t tail = (r + size + kHuge) - (a + size);
    if (tail) munmap((void *)(a + size), tail);
    madvise((void *)a, size, MADV_HUGEPAGE);
    return (void *)a;
}

}  // namespace

void *big_alloc(size_t bytes) {
    const size_t need = (bytes + kHuge - 1) & ~(kHuge - 1);
    Cache &c = cache();
    {
        std::lock_guard<std::mutex> lk(c.mu);
        auto it = c.free_.lower_bound(need);
        if (it != c.free_.end() && it->first <= need + need / 2) {
            void *p = it->second;
            const size_t sz = it->first;
            c.free_.erase(it);
            c.cached -= sz;
            c.live[p] = sz;
            return p;
        }
    }
    void *p = map_block(need);
    std::lock_guard<std::mutex> lk(c.mu);
    c.live[p] = need;
    return p;
}

void big_free(void *p, size_t bytes) noexcept {
    if (!p) return;
    Cache &c = cache();
    std::lock_guard<std::mutex> lk(c.mu);
    auto it = c.live.find(p);
    size_t sz = (bytes + kHuge - 1) & ~(kHuge - 1);
    if (it != c.live.end()) {
        sz = it->second;
        c.live.erase(it);
    }
    c.free_.emplace(sz, p);
    c.cached += sz;
    while (c.cached > kCacheCap && !c.free_.empty()) {   // drop the largest cached blocks first
        auto last = std::prev(c.free_.end());
        unmap_block(last->second, last->first);
        c.cached -= last->first;
        c.free_.erase(last);
    }
}

size_t big_cached_bytes() {
    Cache &c = cache();
    std::lock_guard<std::mutex> lk(c.mu);
    return c.cached;
}

void big_trim() {
    Cache &c = cache();
    std::lock_guard<std::mutex> lk(c.mu);
    for (auto &kv : c.free_) unmap_block(kv.second, kv.first);
    c.free_.clear();
    c.cached = 0;
}

size_t big_block_size(const void *p) {
    Cache &c = cache();
    std::lock_guard<std::mutex> lk(c.mu);
    auto it = c.live.find(const_cast<void *>(p));
    return it == c.live.end() ? 0 : it->second;
}

void big_set_unmap_hook(void (*hook)(void *, size_t)) {
    Cache &c = cache();
    std::lock_guard<std::mutex> lk(c.mu);
    g_unmap_hook = hook;
}

namespace {
class Reaper {
public:
    static Reaper &get() {
        static Reaper r;
        return r;
    }
    void push(std::function<void()> fn) {
        {
            std::lock_guard<std::mutex> lk(mu);
            if (!th.joinable()) th = std::thread([this] { loop(); });
            q.push_back(std::move(fn));
            ++submitted;
        }
        cv.notify_all();
    }
    void drain() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t want = submitted;
        done_cv.wait(lk, [&] { return finished >= want; });
    }
    ~Reaper() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        if (th.joinable()) th.join();   // runs what is still queued first
    }

private:
    void loop() {
        for (;;) {
            std::function<void()> fn;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || !q.empty(); });
                if (q.empty()) return;
                fn = std::move(q.front());
                q.pop_front();
            }
            fn();
            fn = nullptr;
            {
                std::lock_guard<std::mutex> lk(mu);
                ++finished;
            }
            done_cv.notify_all();
        }
    }
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::deque<std::function<void()>> q;
    std::thread th;
    uint64_t submitted = 0, finished = 0;
    bool stop = false;
};
}  // namespace

void defer(std::function<void()> fn) { Reaper::get().push(std::move(fn)); }
void defer_drain() { Reaper::get().drain(); }

}  // namespace bwtmi
