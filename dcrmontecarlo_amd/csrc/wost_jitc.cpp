// wost_jitc -- libwost's compile helper: one field-specialised walk kernel per run.
//
//   wost_jitc [--parent=<pid>] <source file> <code object file> <hiprtc option>...
//   wost_jitc --identity      (prints the hiprtc library it compiles with)
//
// Reads the generated source, compiles it with hiprtc and the given options against the
// headers embedded in this binary (the same bytes as libwost's), writes the code object,
// and exits 0; on a compile error it prints the compiler's log on stderr and exits 1.
// It never touches a GPU: libwost (wost_jit.cpp) starts one per compile so that the
// compiles of concurrent handles overlap, and loads the code object itself. With --parent,
// a helper whose parent process has exited meanwhile (a background compile of a process
// that ended first) removes the scratch directory its files are in.
#include <dirent.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "wost_rtc.h"

int main(int argc, char** argv) {
    if (argc == 2 && std::string(argv[1]) == "--identity") {
        std::printf("%s\n", wost::rtc_library().c_str());
        return 0;
    }
    long parent = -1;
    if (argc > 1 && std::string(argv[1]).rfind("--parent=", 0) == 0) {
        parent = std::atol(argv[1] + 9);
        ++argv;
        --argc;
    }
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s <source file> <code object file> <hiprtc option>...\n", argv[0]);
        return 2;
    }
    std::ifstream in(argv[1], std::ios::binary);
    if (!in) {
        std::fprintf(stderr, "wost_jitc: cannot read %s\n", argv[1]);
        return 2;
    }
    const std::string source((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    std::vector<std::string> options(argv + 3, argv + argc);
    std::vector<char> code;
    std::string log;
    if (!wost::rtc_compile(source, options, &code, &log)) {
        std::fprintf(stderr, "%s\n", log.c_str());
        return 1;
    }
    std::ofstream out(argv[2], std::ios::binary);
    out.write(code.data(), (std::streamsize)code.size());
    out.close();
    if (!out) {
        std::fprintf(stderr, "wost_jitc: cannot write %s\n", argv[2]);
        return 2;
    }
    if (parent > 0 && (long)getppid() != parent) {   // orphaned: nobody will read or remove the files
        std::string dir(argv[1]);
        dir = dir.substr(0, dir.rfind('/'));
        if (DIR* d = opendir(dir.c_str())) {
            while (const dirent* e = readdir(d))
                if (std::string(e->d_name) != "." && std::string(e->d_name) != "..")
                    unlink((dir + "/" + e->d_name).c_str());
            closedir(d);
        }
        rmdir(dir.c_str());
    }
    return 0;
}
