// rt_jit.cpp — compile the scene-specialised render kernel (StaticTrace, scene_codegen.cpp) with hipRTC.
//
// The render body and the per-node helpers are the same source as the offline kernels
// (device/rt_body.h, embedded here as text); only the traversal differs.  Compiled with the same
// numerics flags as the offline build (-ffp-contract=off, correctly rounded f32 div/sqrt), so the
// frames are bit-identical to the generic kernels'.  Modules are cached per (scene, variant, device) in
// the process, and their code objects on disk (cache_dir()) so a new process skips the compile.
#include "rt_jit.h"

#include <hip/hiprtc.h>

#include <dlfcn.h>
#include <fcntl.h>
#include <spawn.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "code_object.h"
#include "device/embedded_headers.inc"
#include "rt_render.h"

namespace rt {
namespace {

struct Entry {
  hipModule_t mod = nullptr;
  JitKernels k;
  bool ok = false;
  std::string why;
};

std::mutex g_mu;
std::map<std::string, std::unique_ptr<Entry>> g_cache;

std::string arch_of(int dev) {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) return "gfx950";
  std::string a = p.gcnArchName;
  size_t c = a.find(':');
  return c == std::string::npos ? a : a.substr(0, c);
}

}  // namespace

// ---- the compiler of the run-time kernels ----------------------------------------------------------------
// A process that imports torch before loading this library (every test, bench.py, smoke()) already holds torch's
// bundled ROCm 7.0 HIP runtime, hipRTC and comgr under the same sonames (libhiprtc.so.7, libamd_comgr.so.3), so the
// hipRTC this library links against resolves to those and compiles with their LLVM 20 (AMD clang 20, roc-7.0.2),
// while a process without torch (bin/raytracing) compiles with /opt/rocm's (ROCm 7.2, AMD clang 22): the same scene
// got different kernels depending on who loaded first.  And LLVM 20 miscompiles the verified sphere walk at its
// 6-wave register budget: its register allocator splits the live ranges of the loop-carried pixel sum (and 12 other
// values) around the camera-ray candidate-list loop and places the split copies at the top of the loop's exit block
// ahead of that block's exec-mask restore (`s_or_b64 exec, exec, s[10:11]`), so only the lanes that ran the loop
// execute them while the inverse copies run for every lane: the other lanes' sums rotate (x, y, z) -> (stale, x, y)
// (profiles/r06_defect/: the LLVM-20 code object with that one instruction moved above the copies is exact,
// LLVM 22's build of the same source is exact).  So the run-time kernels are compiled by rt_jitc, a small program next
// to this library linked against /opt/rocm's hipRTC, started as a child process (posix_spawn; no torch in its address
// space).  (A link namespace of its own — dlmopen of /opt/rocm's libhiprtc — gave the same compiler but crashed
// inside comgr once other libraries had been loaded after it: a second libc in one process.)
// RT_JIT_COMPILER=process (A/B, diagnostics) compiles in this process with the hipRTC it resolved; RT_JITC=<path>
// names another helper.
namespace {
std::string helper_path() {
  if (const char *e = std::getenv("RT_JITC"); e && e[0]) return e;
  Dl_info di;
  if (dladdr(reinterpret_cast<void *>(&helper_path), &di) && di.dli_fname) {
    const std::string p = di.dli_fname;
    const size_t s = p.rfind('/');
    return (s == std::string::npos ? std::string(".") : p.substr(0, s)) + "/rt_jitc";
  }
  return "rt_jitc";
}

// run the helper with `args`; its exit status (-1: it could not be started, -2 - n: killed by signal n)
int run_helper(const std::string &exe, const std::vector<std::string> &args, const std::string &out_file = "") {
  std::vector<char *> argv;
  argv.push_back(const_cast<char *>(exe.c_str()));
  for (const std::string &a : args) argv.push_back(const_cast<char *>(a.c_str()));
  argv.push_back(nullptr);
  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  if (!out_file.empty()) posix_spawn_file_actions_addopen(&fa, 1, out_file.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  pid_t pid = 0;
  const int e = posix_spawn(&pid, exe.c_str(), &fa, nullptr, argv.data(), environ);
  posix_spawn_file_actions_destroy(&fa);
  if (e != 0) return -1;
  int status = 0;
  while (waitpid(pid, &status, 0) < 0)
    if (errno != EINTR) return -1;
  return WIFEXITED(status) ? WEXITSTATUS(status) : WIFSIGNALED(status) ? -2 - WTERMSIG(status) : -1;
}

bool write_file(const std::string &p, const std::string &data) {
  FILE *f = std::fopen(p.c_str(), "wb");
  if (!f) return false;
  const bool ok = std::fwrite(data.data(), 1, data.size(), f) == data.size();
  return (std::fclose(f) == 0) && ok;
}
bool read_file(const std::string &p, std::string *out) {
  FILE *f = std::fopen(p.c_str(), "rb");
  if (!f) return false;
  out->clear();
  char buf[1 << 16];
  for (size_t n; (n = std::fread(buf, 1, sizeof buf, f)) > 0;) out->append(buf, n);
  std::fclose(f);
  return true;
}

struct Compiler {
  bool helper = false;
  std::string exe;
  std::string where;     // "helper:<path>" or "process"
  int major = 0, minor = 0;
};

const Compiler &compiler() {
  static const Compiler c = [] {
    Compiler k;
    const char *mode = std::getenv("RT_JIT_COMPILER");
    if (!(mode && std::strcmp(mode, "process") == 0)) {
      k.exe = helper_path();
      char tmpl[] = "/tmp/rt_jitc_vXXXXXX";
      const int fd = mkstemp(tmpl);
      if (fd >= 0) {
        close(fd);
        std::string v;
        if (access(k.exe.c_str(), X_OK) == 0 && run_helper(k.exe, {"--version"}, tmpl) == 0 && read_file(tmpl, &v) &&
            std::sscanf(v.c_str(), "%d %d", &k.major, &k.minor) == 2) {
          k.helper = true;
          k.where = "helper:" + k.exe;
        }
        std::remove(tmpl);
      }
      if (!k.helper)
        std::fprintf(stderr, "[rt] the kernel compiler %s could not be run: run-time kernels compiled with the process's "
                     "hipRTC\n", k.exe.c_str());
    }
    if (!k.helper) {
      hiprtcVersion(&k.major, &k.minor);
      k.where = "process";
    }
    return k;
  }();
  return c;
}

bool compile_in_process(const std::string &src, const std::vector<std::string> &o, std::vector<char> *code,
                        std::string *log) {
  hiprtcProgram prog;
  const char *hdr_src[] = {kEmbedLayout, kEmbedBody};
  const char *hdr_names[] = {"rt_layout.h", "rt_body.h"};
  if (hiprtcCreateProgram(&prog, src.c_str(), "rt_static.hip", 2, hdr_src, hdr_names) != HIPRTC_SUCCESS) {
    if (log) *log = "hiprtcCreateProgram failed";
    return false;
  }
  std::vector<const char *> opts;
  for (const std::string &x : o) opts.push_back(x.c_str());
  bool ok = hiprtcCompileProgram(prog, static_cast<int>(opts.size()), opts.data()) == HIPRTC_SUCCESS;
  if (log) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    log->assign(n, '\0');
    if (n) hiprtcGetProgramLog(prog, &(*log)[0]);
  }
  if (ok) {
    size_t n = 0;
    hiprtcGetCodeSize(prog, &n);
    code->resize(n);
    ok = n > 0 && hiprtcGetCode(prog, code->data()) == HIPRTC_SUCCESS;
  }
  hiprtcDestroyProgram(&prog);
  return ok;
}

bool compile_in_helper(const std::string &exe, const std::string &src, const std::vector<std::string> &o,
                       std::vector<char> *code, std::string *log) {
  const char *td = std::getenv("TMPDIR");
  std::string tmpl = std::string(td && td[0] ? td : "/tmp") + "/rt_jitc_XXXXXX";
  if (!mkdtemp(&tmpl[0])) {
    if (log) *log = "mkdtemp failed";
    return false;
  }
  const std::string dir = tmpl;
  std::string opts;
  for (const std::string &x : o) opts += x + "\n";
  const char *files[] = {"/src.hip", "/rt_layout.h", "/rt_body.h", "/opts.txt", "/code.co", "/log.txt"};
  bool ok = write_file(dir + files[0], src) && write_file(dir + files[1], kEmbedLayout) &&
            write_file(dir + files[2], kEmbedBody) && write_file(dir + files[3], opts);
  const int rc = ok ? run_helper(exe, {dir}) : 2;
  std::string lg, co;
  read_file(dir + "/log.txt", &lg);
  ok = rc == 0 && read_file(dir + "/code.co", &co) && !co.empty();
  if (log)
    *log = rc == -1 ? "the kernel compiler " + exe + " could not be started"
         : rc < -1  ? "the kernel compiler " + exe + " died of signal " + std::to_string(-2 - rc) + ": " + lg
                    : lg;
  if (ok) code->assign(co.begin(), co.end());
  for (const char *f : files) std::remove((dir + f).c_str());
  rmdir(dir.c_str());
  return ok;
}
}  // namespace

std::string jit_compiler_where() { return compiler().where; }

std::vector<std::string> jit_extra_options() {
  std::vector<std::string> v;
  // RT_JIT_SGPR_MEM=1 (A/B): scalar-register spills go to scratch memory instead of lanes of spill VGPRs
  if (const char *e = std::getenv("RT_JIT_SGPR_MEM"))
    if (e[0] == '1') { v.push_back("-mllvm"); v.push_back("-amdgpu-spill-sgpr-to-vgpr=0"); }
  // RT_JIT_SCHED=<strategy> (A/B): the machine scheduler's strategy (max-ilp, max-memory-clause, iterative-ilp, ...)
  if (const char *e = std::getenv("RT_JIT_SCHED"))
    if (e[0] != '\0') { v.push_back("-mllvm"); v.push_back(std::string("-amdgpu-sched-strategy=") + e); }
  if (const char *e = std::getenv("RT_JIT_OPTS")) {
    std::string cur;
    for (const char *p = e;; ++p) {
      if (*p == ' ' || *p == '\0') {
        if (!cur.empty()) v.push_back(cur);
        cur.clear();
        if (*p == '\0') break;
      } else {
        cur += *p;
      }
    }
  }
  return v;
}

// RT_JIT_WAVES=N asks the register allocator for N waves per SIMD (A/B; default: unconstrained)
std::string waves_attr() {
  if (const char *e = std::getenv("RT_JIT_WAVES"))
    if (std::atoi(e) > 0) return " __attribute__((amdgpu_waves_per_eu(" + std::to_string(std::atoi(e)) + ")))";
  return "";
}

std::string waves_attr_n(int waves);

bool jit_source(const SceneImage &img, int variant, uint32_t max_visits, bool fold, std::string *src, uint32_t *visits,
                bool *folded, int waves) {
  std::string trace;
  if (!generate_static_trace(img, max_visits, fold, &trace, visits, folded)) return false;
  const int v = variant & kJitVarMask;
  const std::string attr = waves_attr_n(waves);
  *src = "#include \"rt_body.h\"\nnamespace rt {\n" + trace +
         "extern \"C\" __global__ __launch_bounds__(256)" + attr + " void rt_static_render(RenderArgs A) {\n"
         "  render_body<" + std::to_string(v | kVarNoProbe) + ", StaticTrace>(A);\n}\n"
         "extern \"C\" __global__ __launch_bounds__(256) void rt_static_render_count(RenderArgs A) {\n"
         "  render_body<" + std::to_string(v | kVarCount | kVarNoProbe) + ", StaticTrace>(A);\n}\n"
         "extern \"C\" __global__ __launch_bounds__(256) void rt_static_probe(RenderArgs A) {\n"
         "  render_body<" + std::to_string(v | kVarProbe) + ", StaticTrace>(A);\n}\n"
         "}  // namespace rt\n";
  return true;
}

// The complete hipRTC option vector.  Same numerics flags as the offline build.  SLP vectorisation is
// off: on this code it packs scalar f32 pairs into v_pk_* with extra moves, turns the planar inside-test
// into a <4 x i1> reduction, and its longer live ranges spill ~100 SGPRs (measured: -10% instructions,
// 86 -> 71 VGPRs on scene 0; measured again in round 1: +30 % frame time).  RT_JIT_OPTS appends options
// (A/B experiments); hipRTC keeps the FIRST of two conflicting flags, so it cannot override these.
// The on-disk cache key hashes this whole vector (build_module): bit-exact parity rests on these flags.
std::vector<std::string> jit_options(const std::string &arch, const std::vector<std::string> &extra) {
  std::vector<std::string> o = {"--offload-arch=" + arch, "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                                "-fhip-fp32-correctly-rounded-divide-sqrt"};
  // RT_JIT_SLP=1 (A/B): let the SLP vectoriser pack f32 pairs into v_pk_* (off by default, above)
  if (const char *e = std::getenv("RT_JIT_SLP"); !(e && e[0] == '1')) o.push_back("-fno-slp-vectorize");
  // Loops are unrolled only where the source asks (#pragma unroll): ROCm 7.2's LLVM 22 otherwise also unrolls the
  // colour-stack unwind and the rejection loops of the scene-specialised kernels (+11 % static VALU instructions, scene 0
  // render +4 % against the LLVM 20 build; without: level, profiles/r06_ab_unroll_*.jsonl).  RT_JIT_UNROLL=1 (A/B)
  // lets the unroller choose.
  if (const char *e = std::getenv("RT_JIT_UNROLL"); !(e && e[0] == '1')) o.push_back("-fno-unroll-loops");
  for (const std::string &x : jit_extra_options()) o.push_back(x);
  for (const std::string &x : extra) o.push_back(x);
  // RT_CHECKS=1: the run-time kernels with device bounds checks (rt_body.h RT_CHECK; diagnostics, debug builds)
  if (const char *e = std::getenv("RT_CHECKS"); e && e[0] == '1') o.push_back("-DRT_DEVICE_CHECKS");
  return o;
}

bool jit_compile(const std::string &src, const std::string &arch, std::vector<char> *code, std::string *log,
                 const std::vector<std::string> &extra) {
  const Compiler &C = compiler();
  const std::vector<std::string> o = jit_options(arch, extra);
  const bool ok = C.helper ? compile_in_helper(C.exe, src, o, code, log) : compile_in_process(src, o, code, log);
  if (ok) {
    if (const char *dir = std::getenv("RT_JIT_DUMP")) {   // diagnostics: source + code object
      const std::string base = std::string(dir) + "/rt_static_" + std::to_string(std::hash<std::string>()(src));
      if (FILE *f = std::fopen((base + ".hip").c_str(), "wb")) { std::fwrite(src.data(), 1, src.size(), f); std::fclose(f); }
      if (FILE *f = std::fopen((base + ".co").c_str(), "wb")) { std::fwrite(code->data(), 1, code->size(), f); std::fclose(f); }
    }
  }
  return ok;
}

namespace {

// ---- on-disk code-object cache -------------------------------------------------------------------
// A fresh process (bin/raytracing, rt_render from a new program) would otherwise pay a hipRTC compile
// (seconds) per scene/variant.  Entries are keyed by everything the code object depends on: the arch,
// the hipRTC version, the extra options, the embedded device headers and the generated source.  The
// full key is stored in the file and compared on load, so a hash collision can only cost a compile.
// Directory: RT_JIT_CACHE_DIR, else $XDG_CACHE_HOME/cuda_raytracing_amd, else ~/.cache/cuda_raytracing_amd;
// RT_JIT_CACHE_DIR=0 disables it.
uint64_t fnv1a(const std::string &s, uint64_t h = 1469598103934665603ull) {
  for (unsigned char ch : s) { h ^= ch; h *= 1099511628211ull; }
  return h;
}

std::string cache_dir() {
  if (const char *e = std::getenv("RT_JIT_CACHE_DIR")) {
    if (e[0] == '\0' || (e[0] == '0' && e[1] == '\0')) return "";
    return e;
  }
  if (const char *x = std::getenv("XDG_CACHE_HOME"); x && x[0]) return std::string(x) + "/cuda_raytracing_amd";
  if (const char *h = std::getenv("HOME"); h && h[0]) return std::string(h) + "/.cache/cuda_raytracing_amd";
  return "";
}

bool make_dirs(const std::string &d) {
  std::string cur;
  for (size_t i = 0; i <= d.size(); ++i) {
    if (i == d.size() || d[i] == '/') {
      if (!cur.empty() && mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return false;
    }
    if (i < d.size()) cur += d[i];
  }
  return true;
}

constexpr char kCacheMagic[8] = {'R', 'T', 'J', 'I', 'T', 'C', 'O', '2'};

bool disk_load(const std::string &path, const std::string &key, std::vector<char> *code) {
  FILE *f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  char magic[8];
  uint64_t klen = 0, clen = 0;
  bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, kCacheMagic, 8) == 0 &&
            std::fread(&klen, 8, 1, f) == 1 && klen == key.size();
  if (ok) {
    std::string k(klen, '\0');
    ok = std::fread(&k[0], 1, klen, f) == klen && k == key && std::fread(&clen, 8, 1, f) == 1 && clen > 0 &&
         clen < (1ull << 30);
    if (ok) {
      code->resize(clen);
      ok = std::fread(code->data(), 1, clen, f) == clen;
    }
  }
  std::fclose(f);
  return ok;
}

void disk_store(const std::string &dir, const std::string &path, const std::string &key, const std::vector<char> &code) {
  if (!make_dirs(dir)) return;
  const std::string tmp = path + ".tmp." + std::to_string(static_cast<long>(getpid()));
  FILE *f = std::fopen(tmp.c_str(), "wb");
  if (!f) return;
  const uint64_t klen = key.size(), clen = code.size();
  bool ok = std::fwrite(kCacheMagic, 1, 8, f) == 8 && std::fwrite(&klen, 8, 1, f) == 1 &&
            std::fwrite(key.data(), 1, klen, f) == klen && std::fwrite(&clen, 8, 1, f) == 1 &&
            std::fwrite(code.data(), 1, clen, f) == clen;
  ok = (std::fclose(f) == 0) && ok;
  if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) std::remove(tmp.c_str());   // atomic publish
}

// Everything outside the source that decides the code object: hipRTC major.minor, the HIP runtime's full
// version (it carries the patch level, i.e. the bundled compiler build), the version this library was
// built against, and the embedded device headers.
std::string toolchain_tag() {
  const int major = compiler().major, minor = compiler().minor;
  int runtime = 0;
  if (hipRuntimeGetVersion(&runtime) != hipSuccess) runtime = -1;
  static const std::string headers = std::to_string(fnv1a(std::string(kEmbedLayout) + '\x01' + kEmbedBody));
  return "hiprtc " + compiler().where + " " + std::to_string(major) + "." + std::to_string(minor) + " runtime " + std::to_string(runtime) +
         " built " + std::to_string(HIP_VERSION_MAJOR) + "." + std::to_string(HIP_VERSION_MINOR) + "." +
         std::to_string(HIP_VERSION_PATCH) + " headers " + headers;
}

// Compile (or fetch) the module of `src` exporting <prefix>_render, <prefix>_render_count, <prefix>_probe.
bool build_module(const std::string &src, const std::string &prefix, JitKernels *out, std::string *why,
                  const std::vector<std::string> &extra = {}) {
  const auto t0 = std::chrono::steady_clock::now();
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  const std::string arch = arch_of(dev);
  std::string opts;
  for (const std::string &x : jit_options(arch, extra)) opts += x + " ";
  const std::string disk_key = arch + "|" + toolchain_tag() + "|" + opts + "|" + src;
  const std::string key = std::to_string(dev) + "|" + disk_key;
  std::lock_guard<std::mutex> lock(g_mu);
  int source = RT_JIT_MEMORY;
  auto it = g_cache.find(key);
  if (it == g_cache.end()) {
    auto e = std::make_unique<Entry>();
    std::vector<char> code;
    std::string log;
    const std::string dir = cache_dir();
    char name[40];
    std::snprintf(name, sizeof name, "/rt_%016llx.co", static_cast<unsigned long long>(fnv1a(disk_key)));
    const std::string path = dir.empty() ? "" : dir + name;
    bool have = !path.empty() && disk_load(path, disk_key, &code);
    source = have ? RT_JIT_DISK : RT_JIT_COMPILED;
    if (!have && jit_compile(src, arch, &code, &log, extra)) {
      have = true;
      if (!path.empty()) disk_store(dir, path, disk_key, code);
    }
    if (!have) {
      e->why = "hipRTC compile failed: " + log.substr(0, 2000);
    } else if ((code_object_kernel(code, prefix + "_render", &e->k.meta_render, &e->k.compiler),
                code_object_kernel(code, prefix + "_render_count", &e->k.meta_count, nullptr),
                hipModuleLoadData(&e->mod, code.data()) != hipSuccess) ||
               hipModuleGetFunction(&e->k.render, e->mod, (prefix + "_render").c_str()) != hipSuccess ||
               hipModuleGetFunction(&e->k.render_count, e->mod, (prefix + "_render_count").c_str()) != hipSuccess ||
               hipModuleGetFunction(&e->k.probe, e->mod, (prefix + "_probe").c_str()) != hipSuccess) {
      e->why = "hipModuleLoadData/GetFunction failed";
    } else {
      e->ok = true;
    }
    it = g_cache.emplace(key, std::move(e)).first;
  }
  if (!it->second->ok) {
    if (why) *why = it->second->why;
    return false;
  }
  const uint32_t visits = out->visits;
  const bool folded = out->folded;
  *out = it->second->k;
  out->visits = visits;
  out->folded = folded;
  out->source = source;
  out->ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return true;
}

}  // namespace


int scene_shading_bits(const SceneImage &img) {
  uint32_t mm = 0, tm = 0;
  for (uint32_t m = 0; m < img.mat_count; ++m) {
    const uint32_t k = img.words[img.off_mats + static_cast<size_t>(m) * kMatWords + M_KIND];
    if (k < 4) mm |= 1u << k;
  }
  for (uint32_t t = 0; t < img.tex_count; ++t) {
    const uint32_t k = img.words[img.off_texs + static_cast<size_t>(t) * kTexWords + T_KIND];
    if (k < 4) tm |= 1u << k;
  }
  if (mm == 0) mm = 15;   // an empty table would read as "all"; keep it explicit
  if (tm == 0) tm = 1u << T_SOLID;
  return static_cast<int>((mm << kVarMatShift) | (tm << kVarTexShift));
}

uint32_t scene_kinds(const SceneImage &img) {
  uint32_t km = 0;
  for (uint32_t i = 0; i < img.node_count; ++i) {
    const uint32_t k = img.words[static_cast<size_t>(i) * kNodeWords + W_KIND];
    if (k < 7) km |= 1u << k;
  }
  return km;
}

std::string jit_lane_source(const SceneImage &img, int variant) {
  const int v = variant & kJitVarMask;
  const std::string lt = "LaneTraceK<" + std::to_string(scene_kinds(img)) + "u, true>";   // pausable walk
  std::string src = "#include \"rt_body.h\"\nnamespace rt {\n";
  src += "extern \"C\" __global__ __launch_bounds__(256) void rt_lane_render(RenderArgs A) {\n  render_body<" +
         std::to_string(v | kVarNoProbe) + ", " + lt + ">(A);\n}\n";
  src += "extern \"C\" __global__ __launch_bounds__(256) void rt_lane_render_count(RenderArgs A) {\n  render_body<" +
         std::to_string(v | kVarCount | kVarNoProbe) + ", " + lt + ">(A);\n}\n";
  src += "extern \"C\" __global__ __launch_bounds__(256) void rt_lane_probe(RenderArgs A) {\n  render_body<" +
         std::to_string(v | kVarProbe) + ", " + lt + ">(A);\n}\n";
  src += "}  // namespace rt\n";
  return src;
}

// RT_JIT_MAX_VGPR=N caps every run-time render kernel at 2N VGPRs (amdgpu_num_vgpr, A/B)
// waves > 0: amdgpu_waves_per_eu(waves); waves < 0: a cap of -waves VGPRs (amdgpu_num_vgpr counts register pairs of
// the unified VGPR/AGPR file on gfx950: N gives 2N VGPRs)
std::string waves_attr_n(int waves) {
  if (waves < 0) return " __attribute__((amdgpu_num_vgpr(" + std::to_string(-waves / 2) + ")))";
  std::string a = waves > 0 ? " __attribute__((amdgpu_waves_per_eu(" + std::to_string(waves) + ")))" : waves_attr();
  if (const char *e = std::getenv("RT_JIT_MAX_VGPR"))
    if (std::atoi(e) > 0) a += " __attribute__((amdgpu_num_vgpr(" + std::to_string(std::atoi(e)) + ")))";
  return a;
}

std::string jit_accel_source(const SceneImage &img, int variant, int waves, int wide) {
  const int v = variant & kJitVarMask;
  const std::string at = "AccelTraceK<" + std::to_string(scene_kinds(img)) + "u, " + (wide ? "true" : "false") + ", " +
                         (wide == 2 ? "true" : "false") + ">";
  std::string src = "#include \"rt_body.h\"\nnamespace rt {\n";
  src += "extern \"C\" __global__ __launch_bounds__(256)" + waves_attr_n(waves) + " void rt_accel_render(RenderArgs A) {\n  render_body<" +
         std::to_string(v | kVarNoProbe) + ", " + at + ">(A);\n}\n";
  src += "extern \"C\" __global__ __launch_bounds__(256) void rt_accel_render_count(RenderArgs A) {\n  render_body<" +
         std::to_string(v | kVarCount | kVarNoProbe) + ", " + at + ">(A);\n}\n";
  src += "extern \"C\" __global__ __launch_bounds__(256) void rt_accel_probe(RenderArgs A) {\n  render_body<" +
         std::to_string(v | kVarProbe) + ", " + at + ">(A);\n}\n";
  src += "}  // namespace rt\n";
  return src;
}

std::string jit_mixed_source(const SceneImage &img, int variant, int waves) {
  const int v = variant & kJitVarMask;
  // pausable walk (RT_MIX_PAUSE=0: the round waits for every walk, A/B)
  const char *pe = std::getenv("RT_MIX_PAUSE");
  const bool pause = !(pe && pe[0] == '0');
  const std::string mt = "MixedTraceK<" + std::to_string(scene_kinds(img)) + "u, " + (pause ? "true" : "false") + ">";
  // the noise octaves one at a time (RT_NOISE_UNROLL, rt_body.h): the unrolled loop's overlapped table reads were the
  // mixed walk's register peak (165 VGPRs, 2 waves; 147 rolled, 3 waves without spilling).  RT_MIX_NOISE_UNROLL (A/B)
  int unroll = 1;
  if (const char *e = std::getenv("RT_MIX_NOISE_UNROLL")) unroll = std::max(1, std::min(7, std::atoi(e)));
  std::string src = "#define RT_NOISE_UNROLL " + std::to_string(unroll) + "\n#include \"rt_body.h\"\nnamespace rt {\n";
  src += "extern \"C\" __global__ __launch_bounds__(256)" + waves_attr_n(waves) + " void rt_mixed_render(RenderArgs A) {\n  render_body<" +
         std::to_string(v | kVarNoProbe) + ", " + mt + ">(A);\n}\n";
  src += "extern \"C\" __global__ __launch_bounds__(256) void rt_mixed_render_count(RenderArgs A) {\n  render_body<" +
         std::to_string(v | kVarCount | kVarNoProbe) + ", " + mt + ">(A);\n}\n";
  src += "extern \"C\" __global__ __launch_bounds__(256) void rt_mixed_probe(RenderArgs A) {\n  render_body<" +
         std::to_string(v | kVarProbe) + ", " + mt + ">(A);\n}\n";
  src += "}  // namespace rt\n";
  return src;
}

// One residency step for a few registers: the allocator often lands just above a boundary of the hardware's
// 16-VGPR granule (the 10k walk at 82 VGPRs = 5 waves/SIMD, 80 would be 6; the mixed walk at 169 = 2, 160 would
// be 3).  When the render kernel is within kRaiseSlack VGPRs of the next residency, its module is rebuilt with
// that residency's register cap (amdgpu_num_vgpr: the waves-per-EU request budgets with an 8-VGPR granule, 168
// for 3 waves, which the hardware's granule does not fit) and kept if the kernel then reaches it with at most
// raise_scratch() bytes of scratch per lane (round 5: none; round 4 kept up to 16 B — the static kernels of scene 0
// and the Cornell box land at 81-87 VGPRs, the mixed walk of final_scene at 169).
// RT_JIT_WAVES (explicit) or RT_JIT_RAISE=0 leaves the first build.
constexpr int kRaiseSlack = 12;
// Scratch a raised build may keep: none by default (round 5).  A build forced under its allocator's register count
// spills VGPRs, and two such builds of the verified sphere walk rendered wrong pixels (and one faulted) where the same
// source at a budget without VGPR spills was exact — each time a small unrelated source edit flipped it.
// RT_JIT_RAISE_SCRATCH=<bytes> (A/B) restores round 4's 16 B.
int raise_scratch() {
  if (const char *e = std::getenv("RT_JIT_RAISE_SCRATCH")) return std::max(0, std::atoi(e));
  return 0;
}

int render_vgprs(hipFunction_t fn, int *scratch) {
  int v = 0, sc = 0;
  if (hipFuncGetAttribute(&v, HIP_FUNC_ATTRIBUTE_NUM_REGS, fn) != hipSuccess) v = 0;
  if (hipFuncGetAttribute(&sc, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, fn) != hipSuccess) sc = -1;
  *scratch = sc;
  return v;
}

// source(n): the module's source with the render kernel's attribute waves_attr_n(n) (n < 0: a cap of -n VGPRs)
template <class Source>
void raise_residency(const Source &source, const char *prefix, JitKernels *out, const std::vector<std::string> &extra = {}) {
  if (std::getenv("RT_JIT_WAVES") || std::getenv("RT_JIT_MAX_VGPR")) return;
  if (const char *e = std::getenv("RT_JIT_RAISE")) if (e[0] == '0') return;
  int sc0 = 0;
  const int v0 = render_vgprs(out->render, &sc0);
  if (v0 <= 0 || sc0 < 0 || sc0 > raise_scratch()) return;
  const int cur = resident_blocks_by_vgprs(v0);
  if (cur >= 8) return;
  const int limit = 512 / (cur + 1) / 16 * 16;   // the hardware's budget for one more wave per SIMD
  if (v0 - limit > kRaiseSlack) return;
  JitKernels k = *out;
  std::string why;
  if (!build_module(source(-limit), prefix, &k, &why, extra)) return;
  int sc = 0;
  const int v = render_vgprs(k.render, &sc);
  if (std::getenv("RT_DEBUG"))
    std::fprintf(stderr, "[rt] jit residency raise %s: %d VGPRs (%d/SIMD) -> cap %d: %d VGPRs, scratch %d B\n",
                 prefix, v0, cur, limit, v, sc);
  if (v > 0 && sc >= 0 && sc <= raise_scratch() && resident_blocks_by_vgprs(v) > cur) {
    k.ms += out->ms;
    *out = k;
  }
}

// Machine-scheduler strategy options: "-amdgpu-sched-strategy=max-ilp" when `on`, unless the environment variable `env`
// names another strategy (or 0 / default: the compiler's default strategy)
std::vector<std::string> sched_options(const char *env, bool on) {
  std::string s = on ? "max-ilp" : "";
  if (const char *e = std::getenv(env)) s = e;
  if (s.empty() || s == "0" || s == "default") return {};
  return {"-mllvm", "-amdgpu-sched-strategy=" + s};
}

// The scene-specialised kernels: max-ilp except with noise textures.  Built by LLVM 22 (round 6) with loops unrolled
// only where asked, max-ilp took scene 0 from 32.1-32.8 to 31.6-31.9 ms and Cornell from 214-216 to 208-211, while the
// Perlin kernel ran +20 % (99 -> 119-121 ms) (profiles/r06_ab_unroll_*.jsonl; round 5 under LLVM 20: scene 0 level,
// Cornell -5 % on one box, Perlin +23 %).  RT_STATIC_SCHED=<strategy> (A/B) builds them with another.
std::vector<std::string> static_sched(const SceneImage &img) { return sched_options("RT_STATIC_SCHED", !img.has_noise); }

bool jit_kernels(const SceneImage &img, int variant, uint32_t max_visits, bool fold, JitKernels *out, std::string *why) {
  std::string src;
  uint32_t visits = 0;
  bool folded = false;
  if (!jit_source(img, variant, max_visits, fold, &src, &visits, &folded)) {
    if (why) *why = "scene expansion exceeds " + std::to_string(max_visits) + " node visits";
    return false;
  }
  out->visits = visits;
  out->folded = folded;
  const std::vector<std::string> sched = static_sched(img);
  if (!build_module(src, "rt_static", out, why, sched)) return false;
  // one residency step up when the allocator lands just above a boundary (kept only with at most raise_scratch()
  // bytes of scratch per lane: none by default)
  raise_residency([&](int w) {
    std::string s2;
    uint32_t v2 = 0;
    bool f2 = false;
    jit_source(img, variant, max_visits, fold, &s2, &v2, &f2, w);
    return s2;
  }, "rt_static", out, sched);
  return true;
}

// The mixed walk is built with the max-ilp scheduler since round 6: under LLVM 22 it ran final_scene 485.5 / 477.0 /
// 486.5 ms against 488.2 / 500.3 / 497.8 with the default strategy (max-memory-clause level; round 5 under LLVM 20:
// max-ilp level; profiles/r06_ab_mixed_sched.jsonl).  RT_MIXED_SCHED=<strategy> (A/B; 0: the default) builds it with another.
std::vector<std::string> mixed_sched() { return sched_options("RT_MIXED_SCHED", true); }

bool jit_mixed_kernels(const SceneImage &img, int variant, JitKernels *out, std::string *why) {
  out->visits = 0;
  out->folded = false;
  const std::vector<std::string> sched = mixed_sched();
  if (!build_module(jit_mixed_source(img, variant), "rt_mixed", out, why, sched)) return false;
  raise_residency([&](int w) { return jit_mixed_source(img, variant, w); }, "rt_mixed", out, sched);
  return true;
}

// The verified sphere walk is latency-bound (dependent node loads): hipRTC allocates its render kernel
// ~97 VGPRs (4 waves/SIMD); asked for 6 waves (80 VGPRs) it runs the 10k frame 226-231 -> 206-208 ms
// (profiles/r03_ab_jit_waves.jsonl).  RT_ACCEL_WAVES=N overrides (0: the allocator's own choice);
// RT_JIT_WAVES, when set, applies to every run-time kernel instead.  Every width is asked for 6 waves (80 VGPRs), and the
// build is kept only if it spills no VGPR (kAccelWavesScratchMax = 0; else the allocator's build and a spill-free raise):
// twice a 6-wave build that spilled VGPRs rendered wrong pixels where the same source without VGPR spills was exact —
// the 4-wide walk of round 4, and in round 5 the 2-wide walk once the tail-piece hand-out was compiled in (G and B of
// samples in mixed waves, a fault at the full 10k config); with its SGPR spills in scratch the same build was exact.
// Since round 5 the 2-wide walk reaches 80 VGPRs without spilling (the pixel sum parked in the lane's stack, the tail
// priority by ballots, the root through a scalar operand).
int accel_waves(int /*wide*/) {
  if (std::getenv("RT_JIT_WAVES")) return 0;
  if (const char *e = std::getenv("RT_ACCEL_WAVES")) return std::max(0, std::min(8, std::atoi(e)));
  return 6;
}

// Width of the verified sphere walk's tree: 2 (the SAH BVH2) or 4 (its 4-wide collapse, accel::collapse_wide)
int accel_width() {
  if (const char *e = std::getenv("RT_ACCEL_WIDTH")) return std::atoi(e) == 4 ? 4 : 2;
  return 2;
}

// The 4-wide tree quantised (accel::quantize_wide, 64-B nodes; RT_ACCEL_QUANT=1) or as float planes (128-B nodes,
// default): measured on the 10k config, the quantised walk is 15 % slower than the float one
bool accel_quant() {
  if (const char *e = std::getenv("RT_ACCEL_QUANT")) return e[0] != '0';
  return false;
}

// The default request is measured on the plain 10k walk (80 VGPRs at 6 waves, no scratch).  Variants that need more
// registers (noise, image u,v, deep bounces: 125-149 VGPRs) would spill; a default-request build with any scratch is
// replaced by the allocator's own build (+ the residency raise, itself spill-free).  An explicit RT_ACCEL_WAVES is kept
// as built.
constexpr int kAccelWavesScratchMax = 0;   // round 4: 96 B (see accel_waves)

// The verified sphere walk's machine-scheduler strategy: max-ilp (the walk's dependent node loads and slab tests
// scheduled for instruction-level parallelism).  Same box (profiles/r05_ab_s54_*): 10k 193.7 / 193.2 ms vs 210.8 /
// 220.1 with the default strategy, at the same 80 VGPRs without a spill; the static kernels keep the default (Perlin
// +23 % under max-ilp, scene 0 level).  RT_ACCEL_SCHED=<strategy> overrides, RT_ACCEL_SCHED=0 keeps the default.
std::vector<std::string> accel_sched() { return sched_options("RT_ACCEL_SCHED", true); }

bool accel_waves_build_kept(int scratch_bytes) { return scratch_bytes >= 0 && scratch_bytes <= kAccelWavesScratchMax; }

bool jit_build_meta(const std::string &src, const std::string &prefix, const std::vector<std::string> &extra,
                    const std::string &arch, KernelMeta *m, std::string *compiler, std::string *why) {
  std::vector<char> code;
  std::string log;
  if (!jit_compile(src, arch, &code, &log, extra)) {
    if (why) *why = "hipRTC compile failed: " + log.substr(0, 2000);
    return false;
  }
  if (!code_object_kernel(code, prefix + "_render", m, compiler)) {
    if (why) *why = "no " + prefix + "_render in the code object's metadata";
    return false;
  }
  return true;
}

bool jit_accel_kernels(const SceneImage &img, int variant, int wide, JitKernels *out, std::string *why) {
  out->visits = 0;
  out->folded = false;
  int w = accel_waves(wide);
  const std::vector<std::string> sched = accel_sched();
  if (!build_module(jit_accel_source(img, variant, w, wide), "rt_accel", out, why, sched)) return false;
  if (w > 0 && !std::getenv("RT_ACCEL_WAVES")) {
    int sc = 0;
    render_vgprs(out->render, &sc);
    if (std::getenv("RT_DEBUG"))
      std::fprintf(stderr, "[rt] jit accel waves_per_eu(%d): scratch %d B per lane\n", w, sc);
    if (!accel_waves_build_kept(sc)) {
      JitKernels k = *out;
      if (!build_module(jit_accel_source(img, variant, 0, wide), "rt_accel", &k, why, sched)) return false;
      k.ms += out->ms;
      *out = k;
      w = 0;
    }
  }
  if (w == 0) raise_residency([&](int n) { return jit_accel_source(img, variant, n, wide); }, "rt_accel", out, sched);
  return true;
}

bool jit_lane_kernels(const SceneImage &img, int variant, JitKernels *out, std::string *why) {
  out->visits = 0;
  out->folded = false;
  return build_module(jit_lane_source(img, variant), "rt_lane", out, why);
}

hipError_t jit_launch(hipFunction_t fn, const RenderArgs &a, uint32_t blocks, size_t lds_bytes, hipStream_t s) {
  RenderArgs copy = a;
  void *args[] = {&copy};
  return hipModuleLaunchKernel(fn, blocks, 1, 1, kBlock, 1, 1, static_cast<unsigned>(lds_bytes), s, args, nullptr);
}

int jit_blocks_per_cu(hipFunction_t fn, size_t lds_bytes) {
  int n = 0;
  if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kBlock, lds_bytes) != hipSuccess || n <= 0) n = 1;
  int vgprs = 0;
  const hipError_t e = hipFuncGetAttribute(&vgprs, HIP_FUNC_ATTRIBUTE_NUM_REGS, fn);
  const int api = n;
  const char *ge = std::getenv("RT_VGPR_GRANULE");   // A/B: 8 = the occupancy table's granule
  if (e == hipSuccess) n = std::min(n, resident_blocks_by_vgprs(vgprs, ge ? std::atoi(ge) : 16));
  if (std::getenv("RT_DEBUG"))
    std::fprintf(stderr, "[rt] jit occupancy: api %d blocks/CU, NUM_REGS %d (%s) -> %d, lds %zu B\n", api, vgprs,
                 hipGetErrorString(e), n, lds_bytes);
  return std::max(n, 1);
}

}  // namespace rt
