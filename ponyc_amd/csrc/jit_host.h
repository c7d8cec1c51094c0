// jit_host.h — behaviours as programs compiled at run time (host side).
//
// The reference compiles every actor type's dispatch: ponyc generates a
// switch over the type's behaviours (src/libponyc/codegen/gentype.c:358-395)
// whose cases destructure the message and call the behaviour's code
// (genfun.c:366-430). A GPU_ACTOR_HT_PROGRAM type brings its behaviours at
// run time as instruction words (include/gpu_actor.h); the device
// interpreter (engine_dev.h) decodes them per message, with its 16 registers
// in scratch. Here the engine does what ponyc does, at run time: each
// program becomes C++ — one function per type, registers as locals, every
// instruction a statement with its label, jumps as gotos — the k_step of
// zone_dev.h is instantiated with it (handler table kHtJit) through hiprtc,
// and the code object is loaded as a module. Results are the interpreter's
// instruction for instruction (an op or pc it ends a behaviour at ends it
// here; a program with a backward jump counts its steps up to
// GPU_ACTOR_PROG_MAX_STEPS); programs hiprtc rejects stay on the
// interpreter. Compiled code objects are cached by a hash of their source:
// in memory for the process, and on disk (GPU_ACTOR_JIT_CACHE, default
// $TMPDIR/gpu_actor_jit).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <dlfcn.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/gpu_actor.h"

namespace jit {

// the device headers, embedded at build time (ponyc_amd/build.py)
#include "jit_headers.inc"

struct Prog {
  uint32_t type;
  std::vector<uint64_t> code;
};

constexpr uint32_t kMaxWords = 1u << 16;    // longer programs stay on the interpreter

inline std::string imm_lit(int64_t v)
{
  return "((uint64_t)(int64_t)(" + std::to_string(v) + "LL))";
}

// One type's behaviours as a device function: the interpreter's loop
// (engine_dev.h handle<GPU_ACTOR_HT_PROGRAM>) unrolled over the program.
inline std::string prog_function(const Prog& p)
{
  const std::vector<uint64_t>& P = p.code;
  const uint32_t np = (uint32_t)P.size();
  const std::string L = "L" + std::to_string(p.type) + "_";
  // a backward jump (a loop) — or more instructions than the step limit —
  // needs the interpreter's step count
  bool count = np > GPU_ACTOR_PROG_MAX_STEPS;
  for(uint32_t pc = 0; pc < np; ++pc)
  {
    const uint32_t op = (uint32_t)P[pc] & 0xFFu;
    const int64_t imm = (int32_t)(uint32_t)(P[pc] >> 32);
    if((op == GPU_ACTOR_OP_JZ || op == GPU_ACTOR_OP_JNZ || op == GPU_ACTOR_OP_JMP) &&
       (int64_t)pc + 1 + imm <= (int64_t)pc)
      count = true;
  }
  std::string s;
  s += "template <class A>\n__device__ __forceinline__ void jit_prog_" + std::to_string(p.type) +
       "(const TypeDev& T, A& a, uint64_t (&s)[8], uint32_t beh, uint64_t arg)\n{\n";
  s += "  uint64_t r0 = s[0], r1 = s[1], r2 = s[2], r3 = s[3], r4 = s[4], r5 = s[5], r6 = s[6], "
       "r7 = s[7];\n";
  s += "  uint64_t r8 = arg, r9 = (uint64_t)a.self, r10 = beh, r11 = 0, r12 = 0, r13 = 0, r14 = 0, "
       "r15 = 0;\n";
  if(count) s += "  uint32_t steps = 0;\n";
  s += "  switch(beh & 15u)\n  {\n";
  for(uint32_t b = 0; b < GPU_ACTOR_PROG_ENTRIES; ++b)
  {
    const uint64_t e = P[b];
    if(e != 0 && e < np) s += "    case " + std::to_string(b) + ": goto " + L + std::to_string(e) + ";\n";
  }
  s += "    default: goto " + L + "end;\n  }\n";
  auto reg = [](uint32_t r) { return "r" + std::to_string(r); };
  for(uint32_t pc = 0; pc < np; ++pc)
  {
    const uint64_t ins = P[pc];
    const uint32_t op = (uint32_t)ins & 0xFFu, d = ((uint32_t)ins >> 8) & 15u;
    const uint32_t ra = ((uint32_t)ins >> 12) & 15u, rb = ((uint32_t)ins >> 16) & 15u;
    const int64_t imm = (int32_t)(uint32_t)(ins >> 32);
    const std::string x = reg(ra), y = reg(rb), D = reg(d);
    s += L + std::to_string(pc) + ":\n";
    if(count) s += "  if(steps >= " + std::to_string(GPU_ACTOR_PROG_MAX_STEPS) + "u) goto " + L + "end;\n  ++steps;\n";
    auto target = [&](void) {
      const int64_t t = (int64_t)pc + 1 + imm;
      return (t < 0 || t >= (int64_t)np) ? L + "end" : L + std::to_string((uint64_t)t);
    };
    switch(op)
    {
      case GPU_ACTOR_OP_LDI:   s += "  " + D + " = " + imm_lit(imm) + ";\n"; break;
      case GPU_ACTOR_OP_LDP:   s += "  " + D + " = T.params[" + std::to_string(imm & 7) + "];\n"; break;
      case GPU_ACTOR_OP_MOV:   s += "  " + D + " = " + x + ";\n"; break;
      case GPU_ACTOR_OP_ADD:   s += "  " + D + " = " + x + " + " + y + ";\n"; break;
      case GPU_ACTOR_OP_SUB:   s += "  " + D + " = " + x + " - " + y + ";\n"; break;
      case GPU_ACTOR_OP_MUL:   s += "  " + D + " = " + x + " * " + y + ";\n"; break;
      case GPU_ACTOR_OP_MULHI: s += "  " + D + " = __umul64hi(" + x + ", " + y + ");\n"; break;
      case GPU_ACTOR_OP_AND:   s += "  " + D + " = " + x + " & " + y + ";\n"; break;
      case GPU_ACTOR_OP_OR:    s += "  " + D + " = " + x + " | " + y + ";\n"; break;
      case GPU_ACTOR_OP_XOR:   s += "  " + D + " = " + x + " ^ " + y + ";\n"; break;
      case GPU_ACTOR_OP_SHL:   s += "  " + D + " = " + x + " << (" + y + " & 63u);\n"; break;
      case GPU_ACTOR_OP_SHR:   s += "  " + D + " = " + x + " >> (" + y + " & 63u);\n"; break;
      case GPU_ACTOR_OP_ADDI:  s += "  " + D + " = " + x + " + " + imm_lit(imm) + ";\n"; break;
      case GPU_ACTOR_OP_LTU:   s += "  " + D + " = " + x + " < " + y + " ? 1ull : 0ull;\n"; break;
      case GPU_ACTOR_OP_EQ:    s += "  " + D + " = " + x + " == " + y + " ? 1ull : 0ull;\n"; break;
      case GPU_ACTOR_OP_MIX:   s += "  " + D + " = splitmix_mix(" + x + ");\n"; break;
      case GPU_ACTOR_OP_JZ:    s += "  if(" + x + " == 0) goto " + target() + ";\n"; break;
      case GPU_ACTOR_OP_JNZ:   s += "  if(" + x + " != 0) goto " + target() + ";\n"; break;
      case GPU_ACTOR_OP_JMP:   s += "  goto " + target() + ";\n"; break;
      case GPU_ACTOR_OP_SEND:
        s += "  if(" + x + " < (uint64_t)c_eng.n_ids) send_serial(a, (uint32_t)" + x + ", " +
             std::to_string((uint32_t)imm & 15u) + "u, " + y +
             ");\n  else atomicAdd(&c_eng.stats[ST_DROPPED], 1ull);\n";
        break;
      case GPU_ACTOR_OP_YIELD: s += "  actor_yield(a);\n"; break;
      case GPU_ACTOR_OP_SPAWN:
        if(((uint32_t)imm & 0xFFu) < GPU_ACTOR_MAX_TYPES)
          s += "  spawn_actor(a, " + std::to_string((uint32_t)imm & 0xFFu) + "u, " +
               std::to_string(((uint32_t)imm >> 8) & 15u) + "u, " + y + ");\n";
        else
          s += "  atomicAdd(&c_eng.stats[ST_DROPPED], 1ull);\n";
        break;
      default:                 // GPU_ACTOR_OP_HALT, an unknown op
        s += "  goto " + L + "end;\n";
        break;
    }
  }
  s += L + "end:\n";
  s += "  s[0] = r0; s[1] = r1; s[2] = r2; s[3] = r3; s[4] = r4; s[5] = r5; s[6] = r6; s[7] = r7;\n";
  s += "  (void)r8; (void)r9; (void)r10; (void)r11; (void)r12; (void)r13; (void)r14; (void)r15;\n}\n\n";
  return s;
}

// The translation unit hiprtc compiles: zone_dev.h's k_step instantiated
// with handler table kHtJit, whose handle() dispatches on the actor's type.
inline std::string unit_source(const std::vector<Prog>& progs, bool z12)
{
  std::string s = "// generated by engine.hip jit (jit_host.h)\n#define GPA_STEP_TU 1\n";
  bool yields = false;
  for(const Prog& p : progs)
    for(size_t k = 0; k < p.code.size(); ++k)       // (a jump may run the entry words too)
      yields |= (p.code[k] & 0xFFu) == GPU_ACTOR_OP_YIELD;
  s += std::string("#define GPA_JIT_YIELD ") + (yields ? "1" : "0") + "\n";
  if(z12)
    s += "#define GPA_ZONE_BITS 12\n#define GPA_ZONE_THREADS 1024\n#define GPA_IDX_CAP 24576\n"
         "#define GPA_TILE 7168\n";
  s += "#include \"zone_dev.h\"\nnamespace gpa {\n";
  for(const Prog& p : progs) s += prog_function(p);
  s += "template <class A>\n__device__ __forceinline__ void handle(HtTag<kHtJit>, const TypeDev& T, A& a,\n"
       "  uint64_t (&s)[8], uint32_t beh, uint64_t arg)\n{\n  switch(a.type)\n  {\n";
  for(const Prog& p : progs)
    s += "    case " + std::to_string(p.type) + ": jit_prog_" + std::to_string(p.type) +
         "(T, a, s, beh, arg); break;\n";
  s += "    default: break;\n  }\n}\n";
  s += "template __global__ void k_step<kHtJit, 1>(uint32_t, uint32_t, uint32_t);\n";
  s += "template __global__ void k_step<kHtJit, 2>(uint32_t, uint32_t, uint32_t);\n}\n";
  return s;
}

// The any-mix step for one mix of compiled tables (`mask`: bit per table
// id): zone_dev.h's any-mix kernel (k_step<-1, 0>) with only those tables'
// drains compiled in (GPA_MIX_MASK) — the full any-mix kernel holds every
// table's, and spills thousands of registers for them.
inline std::string mix_source(uint32_t mask, bool z12)
{
  std::string s = "// generated by engine.hip jit (jit_host.h)\n#define GPA_STEP_TU 1\n";
  s += "#define GPA_MIX_MASK " + std::to_string(mask) + "u\n";
  if(z12)
    s += "#define GPA_ZONE_BITS 12\n#define GPA_ZONE_THREADS 1024\n#define GPA_IDX_CAP 24576\n"
         "#define GPA_TILE 7168\n";
  s += "#include \"zone_dev.h\"\nnamespace gpa {\n"
       "template __global__ void k_step<-1, 0>(uint32_t, uint32_t, uint32_t);\n}\n";
  return s;
}

struct Module {
  hipModule_t mod = nullptr;
  // programs: k_step<kHtJit, 1>, <kHtJit, 2>; a mix: k_step<-1, 0>, none
  hipFunction_t plan = nullptr, rest = nullptr;
  hipDeviceptr_t types = nullptr, eng = nullptr;  // the module's c_types, c_eng
  size_t types_sz = 0, eng_sz = 0;
  int static_lds = 0;
  uint64_t key = 0;
};

inline uint64_t fnv1a(const std::string& s, uint64_t h = 0xcbf29ce484222325ull)
{
  for(unsigned char c : s) { h ^= c; h *= 0x100000001b3ull; }
  return h;
}

// GPU_ACTOR_JIT_CACHE; else jit_cache/ beside the library when that is
// writable (the code objects then travel with the library's tree); else
// $TMPDIR/gpu_actor_jit
inline std::string cache_dir()
{
  const char* d = getenv("GPU_ACTOR_JIT_CACHE");
  if(d && *d) return d;
  Dl_info info;
  if(dladdr(reinterpret_cast<void*>(&cache_dir), &info) && info.dli_fname)
  {
    std::string lib = info.dli_fname;
    const size_t slash = lib.rfind('/');
    if(slash != std::string::npos)
    {
      const std::string dir = lib.substr(0, slash);
      if(access(dir.c_str(), W_OK) == 0) return dir + "/jit_cache";
    }
  }
  const char* t = getenv("TMPDIR");
  return std::string(t && *t ? t : "/tmp") + "/gpu_actor_jit";
}

// A unit's cache key: its source (which holds the programs), the device
// headers it includes and the target
inline uint64_t key_of(const std::string& src, const std::string& arch)
{
  uint64_t h = 0xcbf29ce484222325ull;
  for(const char* hdr : kJitHeaders) h = fnv1a(hdr, h);
  return fnv1a(arch, fnv1a(src, h));
}

// The code object for `src` (compiled, or from a cache); "" on failure.
inline std::string code_object(const std::string& src, const std::string& arch, uint64_t key,
  std::string& log)
{
  static std::mutex mu;
  static std::map<uint64_t, std::string> mem;
  std::lock_guard<std::mutex> lk(mu);
  auto it = mem.find(key);
  if(it != mem.end()) return it->second;
  char name[32];
  snprintf(name, sizeof(name), "%016llx", (unsigned long long)key);
  const std::string dir = cache_dir(), path = dir + "/" + name + ".co";
  if(FILE* f = fopen(path.c_str(), "rb"))
  {
    std::string co;
    char buf[1 << 16];
    size_t n;
    while((n = fread(buf, 1, sizeof(buf), f)) > 0) co.append(buf, n);
    fclose(f);
    if(!co.empty()) return mem[key] = co;
  }
  const int nh = (int)(sizeof(kJitHeaders) / sizeof(kJitHeaders[0]));
  hiprtcProgram prog;
  if(hiprtcCreateProgram(&prog, src.c_str(), "gpu_actor_jit.cu", nh, kJitHeaders, kJitHeaderNames) !=
     HIPRTC_SUCCESS)
  {
    log = "hiprtcCreateProgram failed";
    return "";
  }
  const std::string arch_opt = "--offload-arch=" + arch;
  const char* opts[] = {arch_opt.c_str(), "-O3", "-std=c++17", "-Wno-unused-label"};
  const hiprtcResult rc = hiprtcCompileProgram(prog, 4, opts);
  size_t ls = 0;
  if(hiprtcGetProgramLogSize(prog, &ls) == HIPRTC_SUCCESS && ls > 1)
  {
    std::vector<char> b(ls + 1, 0);
    if(hiprtcGetProgramLog(prog, b.data()) == HIPRTC_SUCCESS) log = b.data();
  }
  std::string co;
  size_t cs = 0;
  if(rc == HIPRTC_SUCCESS && hiprtcGetCodeSize(prog, &cs) == HIPRTC_SUCCESS && cs)
  {
    co.resize(cs);
    if(hiprtcGetCode(prog, &co[0]) != HIPRTC_SUCCESS) co.clear();
  }
  hiprtcDestroyProgram(&prog);
  if(co.empty()) return "";
  // on disk for the next process (written whole, then renamed into place)
  if(mkdir(dir.c_str(), 0755) == 0 || errno == EEXIST)
  {
    const std::string tmp = path + ".tmp" + std::to_string((unsigned long long)getpid());
    if(FILE* f = fopen(tmp.c_str(), "wb"))
    {
      const bool ok = fwrite(co.data(), 1, co.size(), f) == co.size();
      fclose(f);
      if(!ok || rename(tmp.c_str(), path.c_str()) != 0) remove(tmp.c_str());
    }
  }
  return mem[key] = co;
}

// Load the code object of `src` whose kernels are named k1 (and k2): 0, or a
// GPU_ACTOR_E* code (the caller then keeps the compiled-in kernels).
inline int load(const std::string& src, const char* k1, const char* k2, const std::string& arch,
  Module& out, std::string& log)
{
  out = Module{};
  const std::string co = code_object(src, arch, key_of(src, arch), log);
  if(co.empty()) return GPU_ACTOR_EINVAL;
  Module m;
  m.key = key_of(src, arch);
  if(hipModuleLoadData(&m.mod, co.data()) != hipSuccess ||
     hipModuleGetFunction(&m.plan, m.mod, k1) != hipSuccess ||
     (k2 && hipModuleGetFunction(&m.rest, m.mod, k2) != hipSuccess) ||
     hipModuleGetGlobal(&m.types, &m.types_sz, m.mod, "_ZN3gpa7c_typesE") != hipSuccess ||
     hipModuleGetGlobal(&m.eng, &m.eng_sz, m.mod, "_ZN3gpa5c_engE") != hipSuccess)
  {
    (void)hipGetLastError();
    if(m.mod) (void)hipModuleUnload(m.mod);
    log += "\nmodule load failed";
    return GPU_ACTOR_EHIP;
  }
  int a = 0, b = 0;
  if(hipFuncGetAttribute(&a, HIP_FUNC_ATTRIBUTE_SHARED_SIZE_BYTES, m.plan) == hipSuccess &&
     (!m.rest || hipFuncGetAttribute(&b, HIP_FUNC_ATTRIBUTE_SHARED_SIZE_BYTES, m.rest) == hipSuccess))
    m.static_lds = a > b ? a : b;
  else
    m.static_lds = 1 << 30;                           // unknown: never fits
  out = m;
  return 0;
}

// The k_step of these programs, loaded (the kernels' and constants' symbols
// are the names the instantiations lower to: Itanium mangling).
inline int build(const std::vector<Prog>& progs, bool z12, const std::string& arch, Module& out,
  std::string& log)
{
  out = Module{};
  for(const Prog& p : progs)
    if(p.code.size() <= GPU_ACTOR_PROG_ENTRIES || p.code.size() > kMaxWords) return GPU_ACTOR_EINVAL;
  static_assert(gpa::kHtJit == 13, "the mangled names below");
  return load(unit_source(progs, z12), "_ZN3gpa6k_stepILi13ELi1EEEvjjj", "_ZN3gpa6k_stepILi13ELi2EEEvjjj",
              arch, out, log);
}

// The any-mix step of this mix of compiled tables, loaded.
inline int build_mix(uint32_t mask, bool z12, const std::string& arch, Module& out, std::string& log)
{
  return load(mix_source(mask, z12), "_ZN3gpa6k_stepILin1ELi0EEEvjjj", nullptr, arch, out, log);
}

inline void unload(Module& m)
{
  if(m.mod) (void)hipModuleUnload(m.mod);
  m = Module{};
}

} // namespace jit
