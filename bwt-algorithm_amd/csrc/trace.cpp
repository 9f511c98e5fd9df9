// trace.cpp -- roctx ranges around the reference's stages (load, upload, scan,
// index, merge, refine..filter, write; bwt.py:3764-3789, 3892-3944), so a
// `rocprofv3 --marker-trace --kernel-trace` run attributes every kernel and
// every host interval to a stage.  Ranges nest per thread (push/pop); the
// background index build and the unit groups open theirs on their own
// threads.  Without a profiler attached a push/pop is a few ns.
#include <rocprofiler-sdk-roctx/roctx.h>

#include "common.h"

namespace bwtmi {

StageRange::StageRange(const char *name) { roctxRangePushA(name); }
StageRange::~StageRange() { roctxRangePop(); }

}  // namespace bwtmi

extern "C" int bwtmi_trace_push(const char *name) {
    if (!name) return BWTMI_E_ARG;
    roctxRangePushA(name);
    return BWTMI_OK;
}

extern "C" int bwtmi_trace_pop(void) {
    roctxRangePop();
    return BWTMI_OK;
}
