// wost_rtc.h -- the hiprtc driver shared by libwost (in-process compiles) and the
// compile helper wost_jitc (out-of-process compiles, wost_jit.cpp).
//
// ROCm's compiler library serialises the compiles of one process, so a survey whose
// handle threads each need their own field-specialised kernels waited for them one
// after another (C5: 36 kernels, ~21 s before the first survey). libwost therefore runs
// each compile in a child process of its own (wost_jitc, next to libwost.so): the
// threads' compiles overlap, and the code object is the same bytes as an in-process
// compile of the same source and options (tests/test_jit_helper.py).
#pragma once

#include <string>
#include <vector>

namespace wost {

// Compiles `source` (which includes "wost_walk.h") against the embedded headers with
// hiprtc `options` (the target first, --offload-arch=...). On success the code object is
// in *code; on failure false and the compiler's message in *log.
bool rtc_compile(const std::string& source, const std::vector<std::string>& options, std::vector<char>* code,
                 std::string* log);

// The file of the hiprtc library this process compiles with (the loader may have bound
// libwost to another copy than /opt/rocm's: PyTorch-ROCm ships its own, whose compiler is
// another ROCm release's), part of the kernel cache key. wost_jitc --identity prints its own.
std::string rtc_library();

}  // namespace wost
