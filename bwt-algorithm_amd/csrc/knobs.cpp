// knobs.cpp -- the library's run-time switches in one table.  Each is read
// once from the environment variable BWTMI_<NAME> (absent: the default) and
// can be changed in-process through bwtmi_knob_set (the tests flip the
// alternate kernels and the host paths without a new process).  Every knob is
// listed, with what it selects, in INTEGRATION.md "Run-time switches".
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <string>

#include "common.h"

namespace bwtmi {

std::atomic<int64_t> g_knobs[KN_COUNT];

namespace {

struct KnobDef {
    const char *name;
    int64_t def;
};
// order = enum Knob (common.h)
constexpr KnobDef kDefs[KN_COUNT] = {
    {"RUNS_DENSE", 0},          {"RUNS_UNTILED", 0},     {"SA_SMALL", 1},       {"SEG_LEVELS", 1},
    {"SCREEN_WIDE", 0},         {"FM_BYTES", 0},         {"LS_CAP", -1},        {"HOST_SCREEN", 0},
    {"NO_PLAIN", 0},            {"INDEX_LANES", 4},      {"SCAN_LANES", 4},     {"NO_AVX512", 0},
    {"POOL_SPIN_US", -1},       {"UNIT_GROUP_THREADS", 4}, {"STATS", 0},        {"NUMA_BIND", 0},
    {"NUMA_SMT", 0},            {"FAIL_MERGE_CHUNK", -1}, {"HIST_S", 0},         {"DEVICE_CHECKS", 0},
    {"SCREEN_DROP", 1},
};


// filled from the environment when the library is loaded
struct Init {
    Init() {
        for (int k = 0; k < KN_COUNT; ++k) {
            const std::string var = std::string("BWTMI_") + kDefs[k].name;
            const char *e = std::getenv(var.c_str());
            g_knobs[k].store(e && *e ? std::atoll(e) : kDefs[k].def, std::memory_order_relaxed);
        }
    }
} g_init;

int find(const char *name) {
    if (!name) return -1;
    if (!std::strncmp(name, "BWTMI_", 6)) name += 6;
    for (int k = 0; k < KN_COUNT; ++k)
        if (!std::strcmp(name, kDefs[k].name)) return k;
    return -1;
}

}  // namespace
}  // namespace bwtmi

using namespace bwtmi;

extern "C" int bwtmi_knob_set(const char *name, int64_t value) {
    const int k = find(name);
    if (k < 0) return BWTMI_E_ARG;
    g_knobs[k].store(value, std::memory_order_relaxed);
    return BWTMI_OK;
}

extern "C" int bwtmi_knob_get(const char *name, int64_t *value) {
    const int k = find(name);
    if (k < 0 || !value) return BWTMI_E_ARG;
    *value = g_knobs[k].load(std::memory_order_relaxed);
    return BWTMI_OK;
}

extern "C" int bwtmi_knob_default(const char *name, int64_t *value) {
    const int k = find(name);
    if (k < 0 || !value) return BWTMI_E_ARG;
    *value = kDefs[k].def;
    return BWTMI_OK;
}

extern "C" const char *bwtmi_knob_names(void) {
    static const std::string all = [] {
        std::string s;
        for (int k = 0; k < KN_COUNT; ++k) {
            if (k) s += ',';
            s += kDefs[k].name;
        }
        return s;
    }();
    return all.c_str();
}
