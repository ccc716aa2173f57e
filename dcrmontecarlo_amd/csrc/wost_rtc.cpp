// wost_rtc.cpp -- see wost_rtc.h.
#include "wost_rtc.h"

#include <dlfcn.h>
#include <hip/hiprtc.h>
#include <limits.h>
#include <stdlib.h>

// Header sources embedded at build time (Makefile: wost_embedded.cpp).
extern const char wost_embedded_wost_h[];
extern const char wost_embedded_wost_device_h[];
extern const char wost_embedded_wost_walk_h[];

namespace wost {

std::string rtc_library() {
    Dl_info info;
    if (!dladdr(reinterpret_cast<void*>(&hiprtcCompileProgram), &info) || !info.dli_fname) return "unknown";
    char buf[PATH_MAX];
    return realpath(info.dli_fname, buf) ? std::string(buf) : std::string(info.dli_fname);
}

bool rtc_compile(const std::string& source, const std::vector<std::string>& options, std::vector<char>* code,
                 std::string* log) {
    const char* hdrs[] = {wost_embedded_wost_h, wost_embedded_wost_device_h, wost_embedded_wost_walk_h};
    const char* names[] = {"wost.h", "wost_device.h", "wost_walk.h"};
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, source.c_str(), "wost_walk_jit.hip", 3, hdrs, names) != HIPRTC_SUCCESS) {
        *log = "hiprtcCreateProgram failed";
        return false;
    }
    std::vector<const char*> opts;
    for (const std::string& o : options) opts.push_back(o.c_str());
    const hiprtcResult rc = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
    if (rc != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string text(n + 1, '\0');
        if (n) hiprtcGetProgramLog(prog, &text[0]);
        *log = std::string("hiprtc: ") + hiprtcGetErrorString(rc) + ": " + text.c_str();
        hiprtcDestroyProgram(&prog);
        return false;
    }
    size_t n = 0;
    hiprtcGetCodeSize(prog, &n);
    code->resize(n);
    hiprtcGetCode(prog, code->data());
    hiprtcDestroyProgram(&prog);
    return n > 0;
}

}  // namespace wost
