// spec.hip -- scene-specialised row kernels (rt_ctx_set_option(RT_OPT_SPECIALIZE, 1)).
//
// The generic kernels read the flattened scene (rt_blob.h) from HBM: every hierarchy step, object
// and leaf record is a dependent scalar load, and every branch on a record field (leaf kind,
// transform form, cull kind, filter form) is taken at run time.  A scene is immutable after upload,
// so this file compiles the SAME device code (rt_device.h) once more with the scene's tables as
// constexpr data (RT_SPEC): the hierarchy walk unrolls into nested branches over constant boxes,
// every record field is a literal, and the branches on them fold away.  The arithmetic on ray
// values is unchanged -- the same operations in the same order, -ffp-contract=off, constant folding
// only of values the host computed already -- so the pixels are bit-identical (tests/test_gpu_spec.py).
//
// hipRTC (libhiprtc, ROCm) compiles the program at scene upload; the code object is cached per
// process by the program text's hash, and loaded as a module on the context's device.  Launches
// take a specialised kernel when one matches (k_rows.hip), the generic one otherwise.
#include <dlfcn.h>
#include <hip/hiprtc.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

#include "rt_ctx.h"

namespace {

// The device headers as text (build/spec_headers.inc: raw string literals made by the Makefile).
#include "spec_headers.inc"

// The hipRTC the programs compile with: the ROCm installation's own (ROCM_PATH, default /opt/rocm),
// loaded into a link-map namespace of its own (dlmopen) with the code-object manager (comgr) it
// loads.  In a process that imported PyTorch first, the plain libhiprtc.so.7 / libamd_comgr.so.3
// resolve to the copies PyTorch bundles (ROCm 7.0, LLVM 20), whose codegen of the scene-family
// program came out 3.8x larger (128 VGPRs, 1.4 KB/lane of scratch) and 19x slower than this
// ROCm's (LLVM 22; profiles/r05v_family_compilers.txt).  If the namespace cannot be made, the
// process's hipRTC is used and the kernel info says so.
struct Rtc {
  hiprtcResult (*create)(hiprtcProgram*, const char*, const char*, int, const char* const*, const char* const*);
  hiprtcResult (*compile)(hiprtcProgram, int, const char* const*);
  hiprtcResult (*log_size)(hiprtcProgram, size_t*);
  hiprtcResult (*log)(hiprtcProgram, char*);
  hiprtcResult (*code_size)(hiprtcProgram, size_t*);
  hiprtcResult (*code)(hiprtcProgram, char*);
  hiprtcResult (*destroy)(hiprtcProgram*);
  const char* (*err)(hiprtcResult);
  hiprtcResult (*version)(int*, int*);
  std::string origin;                  // which hipRTC: the kernel info's "compiler" note
};
const Rtc& rtc() {
  static const Rtc r = [] {
    Rtc x;
    const char* root = getenv("ROCM_PATH");
    const std::string path = std::string(root && *root ? root : "/opt/rocm") + "/lib/libhiprtc.so.7";
    void* h = dlmopen(LM_ID_NEWLM, path.c_str(), RTLD_NOW | RTLD_LOCAL);
    auto sym = [&](const char* n) { return h ? dlsym(h, n) : nullptr; };
    if (h && sym("hiprtcCreateProgram") && sym("hiprtcCompileProgram") && sym("hiprtcGetCode")) {
      x.create = (decltype(x.create))sym("hiprtcCreateProgram");
      x.compile = (decltype(x.compile))sym("hiprtcCompileProgram");
      x.log_size = (decltype(x.log_size))sym("hiprtcGetProgramLogSize");
      x.log = (decltype(x.log))sym("hiprtcGetProgramLog");
      x.code_size = (decltype(x.code_size))sym("hiprtcGetCodeSize");
      x.code = (decltype(x.code))sym("hiprtcGetCode");
      x.destroy = (decltype(x.destroy))sym("hiprtcDestroyProgram");
      x.err = (decltype(x.err))sym("hiprtcGetErrorString");
      x.version = (decltype(x.version))sym("hiprtcVersion");
      x.origin = path;
    } else {
      x.create = hiprtcCreateProgram;
      x.compile = hiprtcCompileProgram;
      x.log_size = hiprtcGetProgramLogSize;
      x.log = hiprtcGetProgramLog;
      x.code_size = hiprtcGetCodeSize;
      x.code = hiprtcGetCode;
      x.destroy = hiprtcDestroyProgram;
      x.err = hiprtcGetErrorString;
      x.version = hiprtcVersion;
      x.origin = std::string("the process's libhiprtc (") + (h ? "symbols missing" : dlerror()) + ")";
    }
    int ma = 0, mi = 0;
    if (x.version && x.version(&ma, &mi) == HIPRTC_SUCCESS) x.origin += " " + std::to_string(ma) + "." + std::to_string(mi);
    return x;
  }();
  return r;
}

struct SpecCode {
  std::vector<char> code;              // the linked code object
  double compile_ms = 0.0;
};
std::mutex g_spec_mu;
std::map<uint64_t, std::shared_ptr<SpecCode>> g_spec_cache;

uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char ch : s) { h ^= ch; h *= 1099511628211ull; }
  return h;
}

// constexpr T NAME[] = { bit_cast<T>(words), ... }: the host record's exact bits (padding included).
// vary (a family program): per 4-byte word, 1 = the word differs between the family's members -- it is
// emitted as 0 and read from the scene's own table (rt_device.h RT_REC), and VARY_NAME lists the mask.
template <class T>
void emit_table(std::string& s, const char* type, const char* name, const std::vector<T>& v,
                const std::vector<uint8_t>* vary = nullptr) {
  static_assert(sizeof(T) % 8 == 0, "spec tables are emitted as 64-bit words");
  constexpr size_t W = sizeof(T) / 8;
  char buf[64];
  s += "constexpr ";
  s += type;
  s += " ";
  s += name;
  s += "[] = {\n";
  std::vector<T> rows(v);
  if (rows.empty()) {                  // no zero-length arrays: one zero record, never read (N_* = 0)
    rows.resize(1);
    memset((void*)rows.data(), 0, sizeof(T));
  }
  for (size_t ri = 0; ri < rows.size(); ++ri) {
    uint64_t w[W];
    memcpy(w, &rows[ri], sizeof(T));
    if (vary && !v.empty())
      for (size_t i = 0; i < 2 * W; ++i)
        if ((*vary)[ri * 2 * W + i]) w[i / 2] &= i % 2 ? 0xffffffffull : 0xffffffff00000000ull;
    s += "  __builtin_bit_cast(";
    s += type;
    s += ", SpecRaw<";
    snprintf(buf, sizeof buf, "%zu", W);
    s += buf;
    s += ">{{";
    for (size_t i = 0; i < W; ++i) {
      snprintf(buf, sizeof buf, "%s0x%llxull", i ? "," : "", (unsigned long long)w[i]);
      s += buf;
    }
    s += "}}),\n";
  }
  s += "};\n";
  if (vary) {
    s += "constexpr uint8_t VARY_";
    s += name;
    s += "[] = {";
    if (v.empty()) s += "0";
    for (size_t i = 0; i < vary->size(); ++i) s += (*vary)[i] ? (i ? ",1" : "1") : (i ? ",0" : "0");
    s += "};\n";
  }
}

// ---- scene families (rt_spec_family_register): one program for scenes of the same structure
// The frames of an animation differ in some numbers (an object's centre and transform, a colour)
// and share everything else -- table sizes, the hierarchy, kinds and flags, most parameters.  A
// family program holds the words every member shares as constants and reads the others from the
// rendering scene's own tables (rt_device.h RT_REC), so one hipRTC compile serves every member.
template <class T>
void vary_words(const std::vector<T>& a, const std::vector<T>& b, std::vector<uint8_t>* m) {
  const size_t n = a.size() * sizeof(T) / 4;
  m->resize(n, 0);
  const uint32_t* x = (const uint32_t*)(const void*)a.data();
  const uint32_t* y = (const uint32_t*)(const void*)b.data();
  for (size_t i = 0; i < n; ++i) (*m)[i] |= x[i] != y[i];
}
template <class T>
bool same_except(const std::vector<T>& a, const std::vector<T>& b, const std::vector<uint8_t>& m) {
  if (a.size() != b.size()) return false;
  const uint32_t* x = (const uint32_t*)(const void*)a.data();
  const uint32_t* y = (const uint32_t*)(const void*)b.data();
  for (size_t i = 0; i < a.size() * sizeof(T) / 4; ++i)
    if (!m[i] && x[i] != y[i]) return false;
  return true;
}
template <class T>
bool same_bytes(const std::vector<T>& a, const std::vector<T>& b) {
  return a.size() == b.size() && (a.empty() || memcmp(a.data(), b.data(), a.size() * sizeof(T)) == 0);
}

struct SpecFamily {
  int members = 0;
  rt::FlatScene base;                  // member 0, without its texels
  std::vector<uint8_t> v_obj, v_trav, v_strav, v_leaf, v_light;
  std::string src;                     // the program's prelude
};
std::vector<std::shared_ptr<SpecFamily>> g_families;   // under g_spec_mu; newest last

// Same structure: equal table sizes, flags, hierarchy nodes, CSG nodes, filter programs and
// texture records (the family program holds those as plain constants).
bool same_structure(const rt::FlatScene& a, const rt::FlatScene& b) {
  return a.objects.size() == b.objects.size() && a.trav.size() == b.trav.size() && a.strav.size() == b.strav.size() &&
         a.leaves.size() == b.leaves.size() && a.lights.size() == b.lights.size() && same_bytes(a.nodes, b.nodes) &&
         same_bytes(a.prog, b.prog) && same_bytes(a.textures, b.textures) && a.any_transparent == b.any_transparent &&
         a.shadow_early_out == b.shadow_early_out && a.colour_fast == b.colour_fast && a.ray_chains == b.ray_chains;
}
bool family_member(const SpecFamily& F, const rt::FlatScene& f) {
  return same_structure(F.base, f) && same_except(F.base.objects, f.objects, F.v_obj) &&
         same_except(F.base.trav, f.trav, F.v_trav) && same_except(F.base.strav, f.strav, F.v_strav) &&
         same_except(F.base.leaves, f.leaves, F.v_leaf) && same_except(F.base.lights, f.lights, F.v_light);
}


}  // namespace

namespace rt {

// The program's prelude: the scene's tables as constexpr data, then the device code.  fam: the
// family's program (the words that differ between members zeroed, their masks emitted).
static std::string spec_source(const FlatScene& f, const SpecFamily* fam) {
  std::string s;
  char buf[256];
  s += std::string("// scene-specialised row kernels (spec.hip)\n#define RT_SPEC 1\n") +
       (fam ? "#define RT_SPEC_FAMILY 1\n" : "") + "#define RT_TILE_W " + std::to_string(RT_TILE_W) +
       "\n#include \"rt_blob.h\"\n";
  s += "template <int N> struct SpecRaw { unsigned long long w[N]; };\nnamespace rt_spec {\n";
  snprintf(buf, sizeof buf,
           "constexpr int N_OBJECTS = %d, N_LIGHTS = %d, N_TRAV = %d, N_STRAV = %d, SHADOW_EARLY_OUT = %d;\n",
           (int)f.objects.size(), (int)f.lights.size(), (int)f.trav.size(), (int)f.strav.size(), f.shadow_early_out);
  s += buf;
  emit_table(s, "RtObject", "OBJECTS", f.objects, fam ? &fam->v_obj : nullptr);
  emit_table(s, "RtTrav", "TRAV", f.trav, fam ? &fam->v_trav : nullptr);
  emit_table(s, "RtTrav", "STRAV", f.strav, fam ? &fam->v_strav : nullptr);
  emit_table(s, "RtNode", "NODES", f.nodes);
  emit_table(s, "RtLeaf", "LEAVES", f.leaves, fam ? &fam->v_leaf : nullptr);
  emit_table(s, "RtProg", "PROG", f.prog);
  emit_table(s, "RtLight", "LIGHTS", f.lights, fam ? &fam->v_light : nullptr);
  emit_table(s, "RtTexture", "TEXTURES", f.textures);
  s += "}  // namespace rt_spec\n#include \"rt_device.h\"\n";
  return s;
}

// One kernel of the program: rt_spec_rows_<f64><cal> (the megakernel of the scene's mode) or
// rt_spec_def_<f64><cal> (the deferred-shadow kernel), the generic kernels' exact bodies.
static std::string spec_kernel(int kind, int mode, bool fc, int f64, int cal) {
  static const char* args =
      "(RtDevScene S, int y_first, int band_rows, int band_pitch, int n_rows, int max_depth, uint8_t* __restrict__ out, "
      "size_t stride, const int32_t* __restrict__ order, uint32_t* __restrict__ cost, int rgb)";
  char buf[1024], waves[64];
  // The specialised megakernel runs 4 waves/SIMD (128 VGPRs): its unrolled walks keep more values
  // live than the generic loop, and at the generic reflection kernel's 5 waves (96 VGPRs) it spilled
  // 62 VGPRs; 4 waves measured 4.9 % faster on 4K globes (0.3499 vs 0.3679 ms,
  // profiles/r05e_spec_waves_ab.txt).  Diagnostic builds may set RT_SPEC_WAVES.
#ifndef RT_SPEC_WAVES
#define RT_SPEC_WAVES 4
#endif
  snprintf(waves, sizeof waves, "%d", RT_SPEC_WAVES);
  // stack frames in LDS: 4 waves/SIMD leave 10 KB per one-wave workgroup (the generic kernel's 2
  // frames at 5 waves: 4 KB); RT_SPEC_LDS_FRAMES (diagnostic builds) overrides the mode's default
#ifdef RT_SPEC_LDS_FRAMES
  const int kl = RT_SPEC_LDS_FRAMES;
#else
  const int kl = -1;
#endif
  if (kind == 0)
    snprintf(buf, sizeof buf,
             "extern \"C\" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(%s))) "
             "void rt_spec_rows_%d%d%s {\n  __shared__ double s_frames[rows_lds_doubles<%d, %d>()];\n"
             "  rows_body<%d, %s, %s, %s, %d>(S, y_first, band_rows, band_pitch, n_rows, max_depth, out, stride, order, "
             "cost, rgb, (lds_f64*)s_frames);\n}\n",
             waves, f64, cal, args, mode, kl, mode, f64 ? "true" : "false", cal ? "true" : "false", fc ? "true" : "false", kl);
  else
    snprintf(buf, sizeof buf,
             "extern \"C\" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RT_WAVES_PER_EU_DEFERRED))) "
             "void rt_spec_def_%d%d%s {\n  __shared__ ShadowWin win;\n"
             "  deferred_body<%s, %s, %s, %s>(S, y_first, band_rows, band_pitch, n_rows, max_depth, out, stride, order, "
             "cost, rgb, &win);\n}\n",
             f64, cal, args, f64 ? "true" : "false", cal ? "true" : "false", fc ? "true" : "false",
             mode == RT_MODE_REFL ? "false" : "true");
  return buf;
}

// The kernels a context loads, (kind, f64, cal): kind 0 = the megakernel, 1 = the deferred kernel
// (reflection-only scenes: their tail-bound launches' choice).  RT_OPT_SPECIALIZE 1: the RGBA8 /
// RGB8 product launches (f64 = 0, cal = 0); 2: the f64 and calibration instantiations too (tests:
// every launch of a parity test then runs specialised).  Each kernel is its own program (prelude +
// one kernel): the programs compile in parallel, and the inliner sees one kernel per module.
struct SpecKernel { int kind, f64, cal; };
static std::vector<SpecKernel> spec_kernels(const rt_ctx* c) {
  std::vector<SpecKernel> v;
  const int n = c->spec_on >= 2 ? 2 : 1;
  for (int kind = 0; kind < (c->spec_deferred ? 2 : 1); ++kind)
    for (int f64 = 0; f64 < n; ++f64)
      for (int cal = 0; cal < n; ++cal) v.push_back({kind, f64, cal});
  return v;
}
static std::vector<std::string> spec_programs(const rt_ctx* c) {
  std::vector<std::string> v;
  for (const SpecKernel& k : spec_kernels(c)) v.push_back(c->spec_src + spec_kernel(k.kind, c->spec_mode, c->spec_fc, k.f64, k.cal));
  return v;
}

const char* spec_compiler() { return rtc().origin.c_str(); }

void spec_drop(rt_ctx* c) {
  for (auto& m : c->spec_mods)
    if (m) (void)hipModuleUnload(m);
  memset(c->spec_mods, 0, sizeof c->spec_mods);
  c->spec_mod = nullptr;
  memset(c->spec_rows, 0, sizeof c->spec_rows);
  memset(c->spec_def, 0, sizeof c->spec_def);
}

// hipRTC: the program (with the device headers as named headers), the flags the library's own
// kernels are built with (Makefile HIPFLAGS: -O3, no contraction, no fast-math, MachineLICM off).
static int spec_compile(const std::string& src, SpecCode* out) {
  const char* headers[] = {spec_hdr_rt_device, spec_hdr_rt_blob, spec_hdr_rt_math};
  const char* names[] = {"rt_device.h", "rt_blob.h", "rt_math.h"};
  hiprtcProgram prog;
  const Rtc& R = rtc();
  if (R.create(&prog, src.c_str(), "rt_spec.hip", 3, headers, names) != HIPRTC_SUCCESS)
    return fail(RT_ERR_DEVICE, "hiprtcCreateProgram failed");
  const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                        "-mllvm", "-disable-machine-licm"};
  const auto t0 = std::chrono::steady_clock::now();
#ifdef RT_DIAG_ENV
  // diagnostic builds: RT_SPEC_OPTS appends options (space-separated) for compiler A/B runs
  std::vector<std::string> extra;
  std::vector<const char*> all(opts, opts + sizeof opts / sizeof opts[0]);
  if (const char* e = getenv("RT_SPEC_OPTS")) {
    std::string s(e), w;
    for (size_t i = 0; i <= s.size(); ++i)
      if (i == s.size() || s[i] == ' ') { if (!w.empty()) extra.push_back(w); w.clear(); } else w += s[i];
  }
  for (const std::string& x : extra) all.push_back(x.c_str());
  const hiprtcResult r = R.compile(prog, (int)all.size(), all.data());
#else
  const hiprtcResult r = R.compile(prog, (int)(sizeof opts / sizeof opts[0]), opts);
#endif
  out->compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (r != HIPRTC_SUCCESS) {
    size_t n = 0;
    R.log_size(prog, &n);
    std::string log(n + 1, '\0');
    R.log(prog, &log[0]);
    R.destroy(&prog);
    return fail(RT_ERR_DEVICE, "hipRTC compile of the specialised kernels failed: %s\n%.2000s", R.err(r),
                log.c_str());
  }
  size_t n = 0;
  R.code_size(prog, &n);
  out->code.resize(n);
  R.code(prog, out->code.data());
  R.destroy(&prog);
#ifdef RT_DIAG_ENV
  if (const char* dir = getenv("RT_SPEC_DUMP_DIR")) {     // diagnostic builds: the code object and its text
    char path[512];
    snprintf(path, sizeof path, "%s/spec_%016llx.co", dir, (unsigned long long)fnv1a(src));
    if (FILE* fo = fopen(path, "wb")) { fwrite(out->code.data(), 1, n, fo); fclose(fo); }
    snprintf(path, sizeof path, "%s/spec_%016llx.hip", dir, (unsigned long long)fnv1a(src));
    if (FILE* fo = fopen(path, "wb")) { fwrite(src.data(), 1, src.size(), fo); fclose(fo); }
  }
#endif
  return RT_OK;
}

// The code objects of programs: from the process cache, else compiled in parallel (one thread per
// program; hipRTC is thread-safe) and cached.  *compile_ms = the longest compile (0: all cached).
static int spec_codes(const std::vector<std::string>& srcs, std::vector<std::shared_ptr<SpecCode>>* out,
                      double* compile_ms) {
  out->assign(srcs.size(), nullptr);
  std::vector<uint64_t> h(srcs.size());
  {
    std::lock_guard<std::mutex> lk(g_spec_mu);
    for (size_t i = 0; i < srcs.size(); ++i) {
      h[i] = fnv1a(srcs[i]);
      auto it = g_spec_cache.find(h[i]);
      if (it != g_spec_cache.end()) (*out)[i] = it->second;
    }
  }
  std::vector<std::shared_ptr<SpecCode>> fresh(srcs.size());
  std::vector<int> rc(srcs.size(), RT_OK);
  std::vector<std::string> err(srcs.size());
  std::vector<std::thread> th;
  for (size_t i = 0; i < srcs.size(); ++i) {
    if ((*out)[i]) continue;
    fresh[i] = std::make_shared<SpecCode>();
    th.emplace_back([&, i] {
      rc[i] = spec_compile(srcs[i], fresh[i].get());
      if (rc[i]) err[i] = rt_last_error();      // the thread's own error slot
    });
  }
  for (auto& x : th) x.join();
  *compile_ms = 0.0;
  for (size_t i = 0; i < srcs.size(); ++i)
    if (rc[i]) return fail(rc[i], "%s", err[i].c_str());
  std::lock_guard<std::mutex> lk(g_spec_mu);
  for (size_t i = 0; i < srcs.size(); ++i) {
    if ((*out)[i]) continue;
    *compile_ms = std::max(*compile_ms, fresh[i]->compile_ms);
    (*out)[i] = g_spec_cache.emplace(h[i], fresh[i]).first->second;
  }
  return RT_OK;
}

void spec_program(const FlatScene& f, rt_ctx* c) {
  // The walks unroll over every hierarchy node and leaf, twice (nearest hit, shadows), and the
  // shading over every object: code size and compile time grow with the scene (globes.scene, 6
  // objects and 11 leaves: ~15 k instructions, ~8 s of hipRTC per kernel).  Larger scenes keep the
  // generic kernels (fractal.scene: 171 objects).
  c->spec_fits = f.objects.size() <= RT_SPEC_MAX_OBJECTS && f.leaves.size() <= RT_SPEC_MAX_LEAVES;
  c->spec_mode = !f.any_transparent ? RT_MODE_REFL : f.ray_chains ? RT_MODE_CHAIN : RT_MODE_TREE;
  c->spec_fc = f.colour_fast != 0;
  c->spec_deferred = c->spec_mode == RT_MODE_REFL;
  c->spec_family = 0;
  {                                    // a registered family holding this scene: its program
    std::lock_guard<std::mutex> lk(g_spec_mu);
    for (auto it = g_families.rbegin(); it != g_families.rend(); ++it)
      if (family_member(**it, f)) {
        c->spec_src = (*it)->src;
        c->spec_family = (*it)->members;
        return;
      }
  }
  c->spec_src = spec_source(f, nullptr);
}

int spec_build(rt_ctx* c) {
  spec_drop(c);
  if (c->spec_src.empty() || !c->spec_fits) return RT_OK;   // too large to unroll: the generic kernels
  const std::vector<std::string> srcs = spec_programs(c);
  std::vector<std::shared_ptr<SpecCode>> codes;
  int rc = spec_codes(srcs, &codes, &c->spec_compile_ms);
  if (rc) return rc;
  RT_HIP(hipSetDevice(c->device));
  char name[32];
  const std::vector<SpecKernel> ks = spec_kernels(c);
  for (size_t i = 0; i < ks.size(); ++i) {
    const SpecKernel& k = ks[i];
    RT_HIP(hipModuleLoadData(&c->spec_mods[i], codes[i]->code.data()));
    snprintf(name, sizeof name, k.kind ? "rt_spec_def_%d%d" : "rt_spec_rows_%d%d", k.f64, k.cal);
    RT_HIP(hipModuleGetFunction(k.kind ? &c->spec_def[k.f64][k.cal] : &c->spec_rows[k.f64][k.cal], c->spec_mods[i], name));
  }
  c->spec_mod = c->spec_mods[0];
  c->spec_hash = fnv1a(c->spec_src);
  return RT_OK;
}

}  // namespace rt

// rt_scene_precompile (include/rt_abi.h): the specialised programs of a scene into the process cache,
// no device needed -- a host may compile on a worker thread while it renders with the generic kernels
extern "C" int rt_scene_precompile(const rt_scene* s, double* compile_ms) {
  if (!s) return fail(RT_ERR_INVALID, "null scene");
  rt::FlatScene f;
  int rc = rt::flatten(*s, &f);
  if (rc) return rc;
  rt_ctx tmp;
  tmp.spec_on = 1;
  rt::spec_program(f, &tmp);
  if (!tmp.spec_fits) {
    if (compile_ms) *compile_ms = 0.0;
    return fail(RT_ERR_UNSUPPORTED, "scene of %zu objects / %zu leaves is not specialised (limits %d / %d)",
                f.objects.size(), f.leaves.size(), RT_SPEC_MAX_OBJECTS, RT_SPEC_MAX_LEAVES);
  }
  std::vector<std::shared_ptr<SpecCode>> codes;
  double ms = 0.0;
  rc = rt::spec_codes(rt::spec_programs(&tmp), &codes, &ms);
  if (compile_ms) *compile_ms = ms;
  return rc;
}

// rt_scene_spec_program (include/rt_abi.h): the prelude and every kernel rt_scene_precompile compiles
extern "C" int rt_scene_spec_program(const rt_scene* s, char* buf, size_t cap, size_t* len) {
  if (!s || !len || (cap > 0 && !buf)) return fail(RT_ERR_INVALID, "null argument");
  rt::FlatScene f;
  int rc = rt::flatten(*s, &f);
  if (rc) return rc;
  rt_ctx tmp;
  tmp.spec_on = 2;
  rt::spec_program(f, &tmp);
  std::string text = tmp.spec_src;
  for (const rt::SpecKernel& k : rt::spec_kernels(&tmp)) text += rt::spec_kernel(k.kind, tmp.spec_mode, tmp.spec_fc, k.f64, k.cal);
  *len = text.size();
  if (cap > 0) {
    const size_t n = text.size() < cap - 1 ? text.size() : cap - 1;
    memcpy(buf, text.data(), n);
    buf[n] = 0;
  }
  return RT_OK;
}

// rt_spec_family_register (include/rt_abi.h): specialised programs for n scenes (the frames of an
// animation), one per class of scenes of the same structure and object hierarchy (the frames of
// spinning_globes.scene fall in two: the hierarchy's grouping follows the globes' positions);
// contexts whose scene belongs to a class load its program (spec_program).
static bool same_hierarchy(const std::vector<RtTrav>& a, const std::vector<RtTrav>& b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (a[i].obj != b[i].obj || a[i].skip != b[i].skip) return false;
  return true;
}
extern "C" int rt_spec_family_register(const rt_scene* const* scenes, int32_t n, double* compile_ms) {
  if (!scenes || n < 1) return fail(RT_ERR_INVALID, "no scenes");
  std::vector<std::shared_ptr<SpecFamily>> fams;
  rt::FlatScene f;
  for (int32_t i = 0; i < n; ++i) {
    if (!scenes[i]) return fail(RT_ERR_INVALID, "null scene %d", i);
    int rc = rt::flatten(*scenes[i], &f);
    if (rc) return rc;
    f.texels.clear();
    SpecFamily* F = nullptr;
    for (auto& x : fams)
      if (same_structure(x->base, f) && same_hierarchy(x->base.trav, f.trav) && same_hierarchy(x->base.strav, f.strav)) {
        F = x.get();
        break;
      }
    if (!F) {
      fams.push_back(std::make_shared<SpecFamily>());
      F = fams.back().get();
      F->base = f;
    }
    F->members++;
    vary_words(F->base.objects, f.objects, &F->v_obj);
    vary_words(F->base.trav, f.trav, &F->v_trav);
    vary_words(F->base.strav, f.strav, &F->v_strav);
    vary_words(F->base.leaves, f.leaves, &F->v_leaf);
    vary_words(F->base.lights, f.lights, &F->v_light);
  }
  std::vector<std::string> srcs;
  for (auto& F : fams) {
    rt_ctx tmp;
    tmp.spec_on = 1;
    rt::spec_program(F->base, &tmp);             // mode / clamp form / size limits of the class
    if (!tmp.spec_fits)
      return fail(RT_ERR_UNSUPPORTED, "scenes of %zu objects / %zu leaves are not specialised (limits %d / %d)",
                  F->base.objects.size(), F->base.leaves.size(), RT_SPEC_MAX_OBJECTS, RT_SPEC_MAX_LEAVES);
    F->src = rt::spec_source(F->base, F.get());
    tmp.spec_src = F->src;
    for (std::string& s : rt::spec_programs(&tmp)) srcs.push_back(std::move(s));
  }
  std::vector<std::shared_ptr<SpecCode>> codes;   // every class's programs, compiled in parallel
  double ms = 0.0;
  int rc = rt::spec_codes(srcs, &codes, &ms);
  if (compile_ms) *compile_ms = ms;
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_spec_mu);
  for (auto& F : fams) g_families.push_back(F);
  return RT_OK;
}

// rt_spec_family_clear (include/rt_abi.h): forget every registered family (loaded modules stay)
extern "C" int rt_spec_family_clear(void) {
  std::lock_guard<std::mutex> lk(g_spec_mu);
  g_families.clear();
  return RT_OK;
}
