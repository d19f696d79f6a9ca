// rt_jitc — the run-time kernels' compiler process (rt_jit.cpp jit_compile starts it as a child process).
//
// Linked against /opt/rocm's hipRTC (ROCm 7.2, AMD clang 22) and started without torch in its address space, so the
// compiler that builds the scene-specialised render kernels is the same whatever the calling process loaded first
// (a Python process that imports torch resolves libhiprtc.so.7 / libamd_comgr.so.3 to torch's bundled ROCm 7.0 copies,
// whose LLVM 20 miscompiled the verified sphere walk: DESIGN §2).
//
//   rt_jitc <dir>      compile <dir>/src.hip with the headers <dir>/rt_layout.h, <dir>/rt_body.h and the options of
//                      <dir>/opts.txt (one per line); writes <dir>/code.co and <dir>/log.txt.  Exit 0: compiled,
//                      1: the compile failed (log.txt says why), 2: an input or output file failed.
//   rt_jitc --version  prints hipRTC's "major minor".
#include <hip/hiprtc.h>

#include <cstdio>
#include <fstream>
#include <iterator>
#include <sstream>
#include <string>
#include <vector>

namespace {
bool slurp(const std::string &p, std::string *out) {
  std::ifstream f(p, std::ios::binary);
  if (!f) return false;
  out->assign(std::istreambuf_iterator<char>(f), {});
  return true;
}
bool spit(const std::string &p, const char *data, size_t n) {
  FILE *f = std::fopen(p.c_str(), "wb");
  if (!f) return false;
  const bool ok = std::fwrite(data, 1, n, f) == n;
  return (std::fclose(f) == 0) && ok;
}
}  // namespace

int main(int argc, char **argv) {
  if (argc == 2 && std::string(argv[1]) == "--version") {
    int major = 0, minor = 0;
    hiprtcVersion(&major, &minor);
    std::printf("%d %d\n", major, minor);
    return 0;
  }
  if (argc != 2) {
    std::fprintf(stderr, "usage: rt_jitc <dir> | --version\n");
    return 2;
  }
  const std::string dir = argv[1];
  std::string src, lay, body, opts_text;
  if (!slurp(dir + "/src.hip", &src) || !slurp(dir + "/rt_layout.h", &lay) || !slurp(dir + "/rt_body.h", &body) ||
      !slurp(dir + "/opts.txt", &opts_text))
    return 2;
  std::vector<std::string> opts;
  std::istringstream is(opts_text);
  for (std::string line; std::getline(is, line);)
    if (!line.empty()) opts.push_back(line);
  std::vector<const char *> op;
  for (const std::string &o : opts) op.push_back(o.c_str());
  const char *hs[] = {lay.c_str(), body.c_str()};
  const char *hn[] = {"rt_layout.h", "rt_body.h"};
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "rt_static.hip", 2, hs, hn) != HIPRTC_SUCCESS) {
    const char m[] = "hiprtcCreateProgram failed";
    spit(dir + "/log.txt", m, sizeof m - 1);
    return 1;
  }
  const bool ok = hiprtcCompileProgram(prog, static_cast<int>(op.size()), op.data()) == HIPRTC_SUCCESS;
  size_t n = 0;
  hiprtcGetProgramLogSize(prog, &n);
  std::string log(n, '\0');
  if (n) hiprtcGetProgramLog(prog, &log[0]);
  if (!spit(dir + "/log.txt", log.data(), log.size())) return 2;
  int rc = ok ? 0 : 1;
  if (ok) {
    hiprtcGetCodeSize(prog, &n);
    std::vector<char> code(n);
    if (n == 0 || hiprtcGetCode(prog, code.data()) != HIPRTC_SUCCESS) rc = 1;
    else if (!spit(dir + "/code.co", code.data(), code.size())) rc = 2;
  }
  hiprtcDestroyProgram(&prog);
  return rc;
}
