// compile a render-kernel source with hipRTC exactly as rt_jit.cpp does (same options, embedded headers from files)
#include <hip/hiprtc.h>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>
static std::string slurp(const char *p) { std::ifstream f(p); std::stringstream s; s << f.rdbuf(); return s.str(); }
int main(int argc, char **argv) {
  // rtc <src.hip> <layout.h> <body.h> <out.co> [extra options...]
  std::string src = slurp(argv[1]), lay = slurp(argv[2]), body = slurp(argv[3]);
  const char *hs[] = {lay.c_str(), body.c_str()};
  const char *hn[] = {"rt_layout.h", "rt_body.h"};
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "rt_static.hip", 2, hs, hn) != HIPRTC_SUCCESS) return 2;
  std::vector<std::string> o = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                                "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize"};
  for (int i = 5; i < argc; ++i) o.push_back(argv[i]);
  std::vector<const char *> op;
  for (auto &x : o) op.push_back(x.c_str());
  hiprtcResult r = hiprtcCompileProgram(prog, (int)op.size(), op.data());
  size_t n = 0;
  hiprtcGetProgramLogSize(prog, &n);
  std::string log(n, '\0');
  if (n) hiprtcGetProgramLog(prog, &log[0]);
  if (r != HIPRTC_SUCCESS) { fprintf(stderr, "%s\n", log.c_str()); return 1; }
  hiprtcGetCodeSize(prog, &n);
  std::vector<char> code(n);
  hiprtcGetCode(prog, code.data());
  FILE *f = fopen(argv[4], "wb"); fwrite(code.data(), 1, n, f); fclose(f);
  return 0;
}
