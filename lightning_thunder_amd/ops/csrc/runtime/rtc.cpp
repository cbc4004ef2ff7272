// Native runtime of the hipfuse fusion executor (K1): hiprtc compilation of generated
// gfx950 kernels, a process-wide code-object / function cache, and a launch entry point
// that takes the kernel's packed argument struct as one byte buffer.
//
// Role parity: the reference hands fusion regions to nvFuser's C++ runtime
// (thunder/executors/nvfuserex_impl.py:301-412 build a FusionDefinition and
// fd.execute() JIT-compiles + launches it).  Here Python emits HIP source for the
// region (executors/hipfuse_codegen.py) and this layer turns it into machine code:
//   lta_rtc_compile  : source -> code object (works without a GPU: pure compiler)
//   lta_rtc_load     : code object -> hipFunction_t (needs a GPU)
//   lta_rtc_launch   : hipModuleLaunchKernel with HIP_LAUNCH_PARAM_BUFFER_POINTER
// Compiled functions are cached by a 64-bit key chosen by the caller (hash of the source).
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#define LTA_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

struct Loaded {
  hipModule_t module = nullptr;
  hipFunction_t fn = nullptr;
};

std::mutex g_mu;
std::unordered_map<unsigned long long, Loaded> g_funcs;

void copy_log(const std::string& s, char* log, size_t cap) {
  if (!log || cap == 0) return;
  size_t n = s.size() < cap - 1 ? s.size() : cap - 1;
  std::memcpy(log, s.data(), n);
  log[n] = 0;
}

std::vector<std::string> split_opts(const char* opts) {
  std::vector<std::string> out;
  if (!opts) return out;
  std::string cur;
  for (const char* p = opts; *p; ++p) {
    if (*p == ' ') {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(*p);
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

}  // namespace

// Compiles `src` with hiprtc.  On success *code points to a malloc'ed code object of
// *size bytes (free with lta_rtc_free).  Returns 0 or the hiprtcResult; the compiler log
// is copied into `log`.
LTA_EXPORT int lta_rtc_compile(const char* src, const char* name, const char* opts, void** code, size_t* size, char* log,
                               size_t log_cap) {
  hiprtcProgram prog;
  hiprtcResult r = hiprtcCreateProgram(&prog, src, name, 0, nullptr, nullptr);
  if (r != HIPRTC_SUCCESS) return (int)r;
  std::vector<std::string> o = split_opts(opts);
  std::vector<const char*> argv;
  for (auto& s : o) argv.push_back(s.c_str());
  r = hiprtcCompileProgram(prog, (int)argv.size(), argv.data());
  size_t ls = 0;
  hiprtcGetProgramLogSize(prog, &ls);
  std::string lg(ls, '\0');
  if (ls) hiprtcGetProgramLog(prog, &lg[0]);
  copy_log(lg, log, log_cap);
  if (r != HIPRTC_SUCCESS) {
    hiprtcDestroyProgram(&prog);
    return (int)r;
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  void* buf = std::malloc(cs);
  hiprtcGetCode(prog, (char*)buf);
  hiprtcDestroyProgram(&prog);
  *code = buf;
  *size = cs;
  return 0;
}

LTA_EXPORT void lta_rtc_free(void* code) { std::free(code); }

// Loads a code object and resolves `kernel`; cached under `key` (returns the cached
// function if the key is already present).
LTA_EXPORT int lta_rtc_load(unsigned long long key, const void* code, size_t size, const char* kernel, void** fn_out) {
  (void)size;
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_funcs.find(key);
  if (it != g_funcs.end()) {
    *fn_out = (void*)it->second.fn;
    return 0;
  }
  Loaded l;
  hipError_t e = hipModuleLoadData(&l.module, code);
  if (e != hipSuccess) return (int)e;
  e = hipModuleGetFunction(&l.fn, l.module, kernel);
  if (e != hipSuccess) return (int)e;
  g_funcs[key] = l;
  *fn_out = (void*)l.fn;
  return 0;
}

LTA_EXPORT void* lta_rtc_lookup(unsigned long long key) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_funcs.find(key);
  return it == g_funcs.end() ? nullptr : (void*)it->second.fn;
}

// Launches `fn` with its single by-value argument struct given as raw bytes.
LTA_EXPORT int lta_rtc_launch(void* fn, unsigned gx, unsigned gy, unsigned gz, unsigned bx, unsigned by, unsigned bz,
                              unsigned shmem, hipStream_t stream, void* args, size_t args_size) {
  size_t sz = args_size;
  void* config[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  hipError_t e = hipModuleLaunchKernel((hipFunction_t)fn, gx, gy, gz, bx, by, bz, shmem, stream, nullptr, config);
  return (int)e;
}

LTA_EXPORT int lta_rtc_num_cached() {
  std::lock_guard<std::mutex> g(g_mu);
  return (int)g_funcs.size();
}
