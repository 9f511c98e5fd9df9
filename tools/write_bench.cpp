// write_bench.cpp -- how fast can one process put N bytes into one file on this
// host?  The STRfinder writer's output (55 MB at C3, 7 MB per 12.5 Mbp shard)
// goes to one file, and buffered pwrite() serialises on the file's inode lock
// whatever the thread count.  Modes, each on a file rewritten in place (the
// bench rewrites repeat.tab every step, so its page-cache pages exist):
//   pwrite1   one pwrite of the whole buffer
//   pwriteT   T threads, disjoint ranges, one shared fd
//   mmapT     ftruncate + mmap(MAP_SHARED) + T threads memcpy their ranges
// usage: g++ -O2 -pthread tools/write_bench.cpp -o /tmp/write_bench && /tmp/write_bench DIR [threads]
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <functional>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

using clk = std::chrono::steady_clock;

static double ms_since(clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); }

static void par(int T, const std::function<void(int)> &fn) {
    std::vector<std::thread> th;
    for (int k = 1; k < T; ++k) th.emplace_back(fn, k);
    fn(0);
    for (auto &t : th) t.join();
}

int main(int argc, char **argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp";
    const int T = argc > 2 ? std::atoi(argv[2]) : 16;
    const std::string path = dir + "/write_bench.out";
    for (size_t N : {size_t(7) << 20, size_t(55) << 20}) {
        std::vector<char> buf(N);
        for (size_t i = 0; i < N; ++i) buf[i] = "ACGT\t\n"[(i * 2654435761u >> 7) % 6];
        { int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644); if (pwrite(fd, buf.data(), N, 0) != (ssize_t)N) return 1; close(fd); }
        std::vector<double> a, b, c;
        for (int rep = 0; rep < 7; ++rep) {
            auto t = clk::now();
            int fd = open(path.c_str(), O_WRONLY | O_CREAT, 0644);
            size_t w = 0;
            while (w < N) w += (size_t)pwrite(fd, buf.data() + w, N - w, (off_t)w);
            if (ftruncate(fd, (off_t)N)) return 1;
            close(fd);
            a.push_back(ms_since(t));

            t = clk::now();
            fd = open(path.c_str(), O_WRONLY | O_CREAT, 0644);
            par(T, [&](int k) {
                size_t x = N * k / T;
                const size_t e = N * (k + 1) / T;
                while (x < e) x += (size_t)pwrite(fd, buf.data() + x, e - x, (off_t)x);
            });
            if (ftruncate(fd, (off_t)N)) return 1;
            close(fd);
            b.push_back(ms_since(t));

            t = clk::now();
            fd = open(path.c_str(), O_RDWR | O_CREAT, 0644);
            if (ftruncate(fd, (off_t)N)) return 1;
            char *m = (char *)mmap(nullptr, N, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            if (m == MAP_FAILED) return 1;
            par(T, [&](int k) {
                const size_t x = N * k / T, e = N * (k + 1) / T;
                std::memcpy(m + x, buf.data() + x, e - x);
            });
            munmap(m, N);
            close(fd);
            c.push_back(ms_since(t));
        }
        auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
        std::printf("{\"bytes\": %zu, \"threads\": %d, \"pwrite1_ms\": %.3f, \"pwriteT_ms\": %.3f, \"mmapT_ms\": %.3f, "
                    "\"pwrite1_gbs\": %.2f, \"mmapT_gbs\": %.2f}\n",
                    N, T, med(a), med(b), med(c), N / med(a) / 1e6, N / med(c) / 1e6);
    }
    unlink(path.c_str());
    return 0;
}
