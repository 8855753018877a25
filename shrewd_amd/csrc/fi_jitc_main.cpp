// fi_jitc_main.cpp -- the JIT helper: builds the trial kernels with the
// translated golden blocks in a process of its own (fi_jit.cpp:rtc_build_child).
//
//   fi_jitc SRC OUT [hipRTC options...]
//
// Writes the code object to OUT, or a log to OUT.log and exits 1.  Never
// touches the GPU.
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

namespace fi {
std::string rtc_build(const std::string &src, const std::vector<const char *> &opts, std::vector<char> &code);
}

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    std::ifstream in(argv[1], std::ios::binary);
    const std::string src((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    std::vector<const char *> opts(argv + 3, argv + argc);
    std::vector<char> code;
    const std::string msg = fi::rtc_build(src, opts, code);
    const std::string out = argv[2];
    if (!msg.empty() || code.empty()) {
        std::ofstream log(out + ".log");
        log << (msg.empty() ? std::string("empty code object") : msg);
        return 1;
    }
    std::ofstream o(out + ".tmp", std::ios::binary);
    o.write(code.data(), (std::streamsize)code.size());
    o.close();
    return std::rename((out + ".tmp").c_str(), out.c_str()) == 0 ? 0 : 1;
}
