// spec.hip -- scene-specialised row kernels (rt_ctx_set_option(RT_OPT_SPECIALIZE), default on).
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
// Life of a program (round 5):
//   * rt_ctx_upload REQUESTS the scene's programs and returns at once: a small pool of library
//     threads compiles them with hipRTC (or finds them in the process cache / the on-disk cache),
//     while the context renders with the generic kernels;
//   * the first launch after the compile finished loads the code objects on the context's device and
//     every later launch takes them (k_rows.hip launch_bands -> spec_poll); rt_ctx_spec_wait blocks
//     for them (hosts that want the specialised kernels from their first timed frame, and tests);
//   * a program is keyed by its FULL text (the process cache compares the text, the disk cache the
//     text and the compiler's identity), never by a hash alone;
//   * guards: only the ROCm installation's hipRTC compiles (loaded into a link-map namespace of its
//     own, see rtc()), and a code object whose resource use exceeds the known-good bound (VGPRs,
//     scratch per lane, from the code object's metadata) is refused -- the context then keeps
//     the generic kernels and rt_ctx_kernel_info says why.  A failed compile never fails an upload.
#include <dlfcn.h>
#include <hip/hiprtc.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
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
  bool rocm = false;                   // the ROCm installation's own (the only one the guard lets compile)
  std::string identity;                // origin + the library file's real path, size and mtime (disk-cache key)
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
      x.rocm = true;
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
    x.identity = x.origin;
    if (char* rp = realpath(path.c_str(), nullptr)) {
      struct stat st;
      if (stat(rp, &st) == 0)
        x.identity += std::string(" ") + rp + " " + std::to_string((long long)st.st_size) + " " + std::to_string((long long)st.st_mtime);
      free(rp);
    }
    return x;
  }();
  return r;
}

uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char ch : s) { h ^= ch; h *= 1099511628211ull; }
  return h;
}
std::mutex g_spec_mu;                  // the job table and the registered families

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
  std::vector<std::shared_ptr<rt::SpecJob>> jobs;   // its compiled kernels, kept resident while registered
};
std::vector<std::shared_ptr<SpecFamily>> g_families;   // under g_spec_mu; newest last
std::vector<std::shared_ptr<SpecFamily>> g_singles;    // "families" of one registered scene: hold its own program

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

bool same_structure_flat(const FlatScene& a, const FlatScene& b) { return same_structure(a, b); }

// A diagnostic build's -D switches (Makefile: $(DIAG) as the string RT_SPEC_DIAG_DEFINES) as #define
// lines for the programs' prelude, so the specialised kernels of a diagnostic build are built the way
// its precompiled kernels are (empty in the product build).
#ifndef RT_SPEC_DIAG_DEFINES
#define RT_SPEC_DIAG_DEFINES ""
#endif
static std::string diag_prelude() {
  std::string out, w;
  const std::string s = RT_SPEC_DIAG_DEFINES;
  for (size_t i = 0; i <= s.size(); ++i) {
    if (i < s.size() && s[i] != ' ') { w += s[i]; continue; }
    if (w.rfind("-D", 0) == 0 && w.size() > 2) {
      const size_t eq = w.find('=');
      out += "#define " + (eq == std::string::npos ? w.substr(2) : w.substr(2, eq - 2) + " " + w.substr(eq + 1)) + "\n";
    }
    w.clear();
  }
  return out;
}

// The program's prelude: the scene's tables as constexpr data, then the device code.  fam: the
// family's program (the words that differ between members zeroed, their masks emitted).
static std::string spec_source(const FlatScene& f, const SpecFamily* fam) {
  std::string s;
  char buf[256];
  s += std::string("// scene-specialised row kernels (spec.hip)\n#define RT_SPEC 1\n") + diag_prelude() +
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
// Chain-mode programs (the anim120 families: 82 VGPRs, 6 waves/SIMD set by the VGPRs and the 6 KB of
// LDS frames) at 7 waves (72 VGPRs, 11 spilled, a 100-110-slot pool) measured 0.5-1 % slower
// (profiles/r08j_chain_waves_ab.txt).  Diagnostic builds may set RT_SPEC_WAVES_CHAIN.
#ifndef RT_SPEC_WAVES_CHAIN
#define RT_SPEC_WAVES_CHAIN RT_SPEC_WAVES
#endif
  // The primary-ray kernel: no frame stack, so its VGPRs (not a fixed budget) set its occupancy.
#ifndef RT_SPEC_WAVES_PRIM
#define RT_SPEC_WAVES_PRIM 4
#endif
  snprintf(waves, sizeof waves, "%d", mode == RT_MODE_CHAIN ? RT_SPEC_WAVES_CHAIN : RT_SPEC_WAVES);
  // stack frames in LDS: 4 waves/SIMD leave 10 KB per one-wave workgroup (the generic kernel's 2
  // frames at 5 waves: 4 KB); RT_SPEC_LDS_FRAMES (diagnostic builds) overrides the mode's default
#ifdef RT_SPEC_LDS_FRAMES
  int kl = RT_SPEC_LDS_FRAMES;
#else
  int kl = -1;
#endif
  int kp = -1;                                                  // the wave pool's slots (-1: the mode's default)
#ifdef RT_DIAG_ENV
  if (const char* e = getenv("RT_SPEC_KL")) kl = atoi(e);      // diagnostic builds: A/B of the LDS frames
  if (const char* e = getenv("RT_SPEC_KP")) kp = atoi(e);
#endif
  if (kind == 2)                                              // the primary-ray kernel (rt_device.h PRIM)
    snprintf(buf, sizeof buf,
             "extern \"C\" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(%d))) "
             "void rt_spec_prim_%d%d%s {\n"
             "  rows_body<%d, %s, %s, %s, 0, 0, true>(S, y_first, band_rows, band_pitch, n_rows, 0, out, stride, order, "
             "cost, rgb, nullptr);\n}\n",
             RT_SPEC_WAVES_PRIM, f64, cal, args, mode, f64 ? "true" : "false", cal ? "true" : "false", fc ? "true" : "false");
  else if (kind == 0)
    snprintf(buf, sizeof buf,
             "extern \"C\" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(%s))) "
             "void rt_spec_rows_%d%d%s {\n  __shared__ double s_frames[rows_lds_doubles<%d, %d, %d>()];\n"
             "  rows_body<%d, %s, %s, %s, %d, %d>(S, y_first, band_rows, band_pitch, n_rows, max_depth, out, stride, order, "
             "cost, rgb, (lds_f64*)s_frames);\n}\n",
             waves, f64, cal, args, mode, kl, kp, mode, f64 ? "true" : "false", cal ? "true" : "false", fc ? "true" : "false",
             kl, kp);
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
// (reflection-only scenes: their tail-bound launches' choice), 2 = the primary-ray kernel (launches
// with max_depth 0).  RT_OPT_SPECIALIZE 1: the RGBA8 / RGB8 product launches (f64 = 0, cal = 0); 2: the
// f64 and calibration instantiations too (tests: every launch of a parity test then runs specialised).
// Each kernel is its own program (prelude + one kernel): the programs compile in parallel, and the
// inliner sees one kernel per module.
struct SpecKernel { int kind, f64, cal; };
static std::vector<SpecKernel> spec_kernels(const rt_ctx* c) {
  std::vector<SpecKernel> v;
  const int n = c->spec_on >= 2 ? 2 : 1;
  for (int kind = 0; kind < 3; ++kind) {
    if (kind == 1 && !c->spec_deferred) continue;
    for (int f64 = 0; f64 < n; ++f64)
      for (int cal = 0; cal < n; ++cal) v.push_back({kind, f64, cal});
  }
  return v;
}
static const char* spec_kernel_name(int kind) {
  return kind == 2 ? "rt_spec_prim_%d%d" : kind == 1 ? "rt_spec_def_%d%d" : "rt_spec_rows_%d%d";
}
static std::vector<std::string> spec_programs(const rt_ctx* c) {
  std::vector<std::string> v;
  for (const SpecKernel& k : spec_kernels(c)) v.push_back(c->spec_src + spec_kernel(k.kind, c->spec_mode, c->spec_fc, k.f64, k.cal));
  return v;
}

// ---- programs: the job table and the compile pool -------------------------------------------------
enum { SPEC_QUEUED = 0, SPEC_RUNNING, SPEC_DONE, SPEC_FAILED, SPEC_CANCELLED };

struct SpecCode {
  std::vector<char> code;              // the linked code object
  std::string name;                    // the kernel (code-object metadata .name)
  double compile_ms = 0.0;             // the hipRTC compile that made it (0: read from the disk cache)
  bool from_disk = false;
  int vgprs = -1, sgprs = -1, scratch = -1, vspill = -1, occupancy = -1;   // code-object metadata (occupancy: VGPR-limited)
};

// One program (prelude + one kernel), keyed by its full text.  `interest` counts the holders (contexts,
// registered families, callers waiting for it): a job nobody holds when a worker reaches it is
// cancelled, so a host that uploads scene after scene (the reference's animate mode builds every
// frame's scene anew, gui.rs:78-89) only ever compiles what it still renders.
struct SpecJob {
  std::string text;
  std::atomic<int> state{SPEC_QUEUED};
  std::atomic<int> interest{0};
  SpecCode code;                       // valid once SPEC_DONE
  std::string error;                   // set once SPEC_FAILED
  uint64_t last_use = 0;
  std::mutex mu;
  std::condition_variable cv;
};

}  // namespace rt

namespace {

using rt::SpecCode;
using rt::SpecJob;
using rt::SPEC_QUEUED;
using rt::SPEC_RUNNING;
using rt::SPEC_DONE;
using rt::SPEC_FAILED;
using rt::SPEC_CANCELLED;

// At most this many compiles at once (hipRTC / LLVM: seconds and hundreds of MB each).
constexpr size_t RT_SPEC_WORKERS_MAX = 4;
// Completed programs the process keeps when nobody holds them (LRU beyond this many jobs).
constexpr size_t RT_SPEC_CACHE_JOBS = 64;
// Resource guard: the known-good bounds of the specialised kernels (ROCm 7.2's LLVM: the reflection and
// chain megakernels at most 128 VGPRs at 4 waves/SIMD with 528-576 B/lane of scratch; the ray-tree
// megakernel 1 424 B/lane for its pending-reflection stack, the deferred kernel 1 568 B/lane for its
// per-lane hit records).  PyTorch's bundled LLVM 20 built the chain family megakernel with 1.4 KB/lane
// and ran it 19x slower (profiles/r05v_family_compilers.txt): that is what the guard refuses.
#ifndef RT_SPEC_MAX_VGPRS
#define RT_SPEC_MAX_VGPRS 128
#endif
#ifndef RT_SPEC_MAX_SCRATCH_ROWS
#define RT_SPEC_MAX_SCRATCH_ROWS 1024
#endif
#ifndef RT_SPEC_MAX_SCRATCH_DEF
#define RT_SPEC_MAX_SCRATCH_DEF 2048
#endif
#ifndef RT_SPEC_MAX_SCRATCH_TREE
#define RT_SPEC_MAX_SCRATCH_TREE 2048
#endif

struct SpecState {                     // under g_spec_mu; never destroyed (workers may outlive exit's destructors)
  std::map<std::string, std::shared_ptr<SpecJob>> jobs;   // by full program text
  uint64_t clock = 0;
  std::deque<std::shared_ptr<SpecJob>> queue;
  std::vector<std::thread> workers;
  std::condition_variable qcv;
  bool stop = false;
  std::string disk_dir;                // rt_spec_cache_dir: "" = no on-disk cache
};
SpecState& sst() {
  static SpecState* p = new SpecState;
  return *p;
}

void job_finish(SpecJob* j, int state) {
  {
    std::lock_guard<std::mutex> lk(j->mu);
    j->state = state;
  }
  j->cv.notify_all();
}

// A token of interest in job j: a shared_ptr to the job whose deleter drops the interest again.
std::shared_ptr<SpecJob> job_token(const std::shared_ptr<SpecJob>& j) {
  j->interest++;
  return std::shared_ptr<SpecJob>(j.get(), [j](SpecJob*) { j->interest--; });
}

bool job_finished(const SpecJob* j) {
  const int s = j->state.load();
  return s == SPEC_DONE || s == SPEC_FAILED || s == SPEC_CANCELLED;
}

// Waits for j (timeout_ms < 0: no limit); true once it has finished.
bool job_wait(SpecJob* j, double timeout_ms) {
  std::unique_lock<std::mutex> lk(j->mu);
  if (timeout_ms < 0) {
    j->cv.wait(lk, [&] { return job_finished(j); });
    return true;
  }
  return j->cv.wait_for(lk, std::chrono::duration<double, std::milli>(timeout_ms), [&] { return job_finished(j); });
}

// The kernel's resource use from the code object's AMDGPU metadata note (msgpack): the map entry after
// the key string, e.g. ".vgpr_count" -> 128.  One kernel per program, so every key occurs once.
// (hipRTC's -Rpass-analysis=kernel-resource-usage remarks say the same, but emitting them crashed the
// compiler inside its own link-map namespace.)
bool mp_value(const std::vector<char>& b, const char* key, long long* ival, std::string* sval) {
  const size_t n = strlen(key);
  std::string pat;
  if (n < 32) pat += (char)(0xa0 | n);
  else { pat += (char)0xd9; pat += (char)n; }
  pat += key;
  const auto it = std::search(b.begin(), b.end(), pat.begin(), pat.end());
  if (it == b.end()) return false;
  size_t i = (size_t)(it - b.begin()) + pat.size();
  if (i >= b.size()) return false;
  const unsigned char t = (unsigned char)b[i];
  auto be = [&](int bytes) {
    unsigned long long v = 0;
    for (int k = 1; k <= bytes && i + k < b.size(); ++k) v = v << 8 | (unsigned char)b[i + k];
    return v;
  };
  if (sval) {
    size_t len = 0, at = 0;
    if ((t & 0xe0) == 0xa0) { len = t & 0x1f; at = i + 1; }
    else if (t == 0xd9) { len = (size_t)be(1); at = i + 2; }
    else return false;
    if (at + len > b.size()) return false;
    sval->assign(b.data() + at, len);
    return true;
  }
  if (t <= 0x7f) *ival = t;
  else if (t == 0xcc) *ival = (long long)be(1);
  else if (t == 0xcd) *ival = (long long)be(2);
  else if (t == 0xce) *ival = (long long)be(4);
  else if (t == 0xcf) *ival = (long long)be(8);
  else return false;
  return true;
}
void code_resources(SpecCode* c) {
  long long v = -1;
  c->vgprs = mp_value(c->code, ".vgpr_count", &v, nullptr) ? (int)v : -1;
  c->sgprs = mp_value(c->code, ".sgpr_count", &v, nullptr) ? (int)v : -1;
  c->scratch = mp_value(c->code, ".private_segment_fixed_size", &v, nullptr) ? (int)v : -1;
  c->vspill = mp_value(c->code, ".vgpr_spill_count", &v, nullptr) ? (int)v : -1;
  c->occupancy = c->vgprs > 0 ? std::min(8, 512 / ((c->vgprs + 7) / 8 * 8)) : -1;   // VGPR-limited waves/SIMD
  std::string name;
  c->name = mp_value(c->code, ".name", nullptr, &name) ? name : "";
}

// The hipRTC options: the flags the library's own kernels are built with (Makefile HIPFLAGS: -O3, no
// contraction, no fast-math, MachineLICM off).
std::vector<std::string> spec_options() {
  std::vector<std::string> opts = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                                   "-mllvm", "-disable-machine-licm"};
#ifdef RT_DIAG_ENV
  // diagnostic builds: RT_SPEC_OPTS appends options (space-separated) for compiler A/B runs
  if (const char* e = getenv("RT_SPEC_OPTS")) {
    std::string s(e), w;
    for (size_t i = 0; i <= s.size(); ++i)
      if (i == s.size() || s[i] == ' ') { if (!w.empty()) opts.push_back(w); w.clear(); } else w += s[i];
  }
#endif
  return opts;
}

// The disk-cache identity of a code object: the compiler's (rtc().identity) plus a hash of everything
// else the object depends on besides the program text -- the device headers this library embeds (the
// text only #includes them) and the compile options.  A rebuild that changes a header (a record layout,
// a kernel argument) changes the identity, so an entry written by another build is never read.
std::string spec_build_identity() {
  std::string key;
  for (const char* h : {spec_hdr_rt_device, spec_hdr_rt_blob, spec_hdr_rt_math}) {
    key += h;
    key += '\0';
  }
  for (const std::string& o : spec_options()) {
    key += o;
    key += '\0';
  }
  char buf[40];
  snprintf(buf, sizeof buf, " build %016llx", (unsigned long long)fnv1a(key));
  return rtc().identity + buf;
}

// hipRTC: the program (with the device headers as named headers), spec_options(), and the resource use
// the guard reads from the code object.
int spec_compile(const std::string& src, SpecCode* out, std::string* err) {
  const char* headers[] = {spec_hdr_rt_device, spec_hdr_rt_blob, spec_hdr_rt_math};
  const char* names[] = {"rt_device.h", "rt_blob.h", "rt_math.h"};
  hiprtcProgram prog;
  const Rtc& R = rtc();
  if (R.create(&prog, src.c_str(), "rt_spec.hip", 3, headers, names) != HIPRTC_SUCCESS) {
    *err = "hiprtcCreateProgram failed";
    return RT_ERR_DEVICE;
  }
  const std::vector<std::string> ostr = spec_options();
  std::vector<const char*> opts;
  for (const std::string& x : ostr) opts.push_back(x.c_str());
  const auto t0 = std::chrono::steady_clock::now();
  const hiprtcResult r = R.compile(prog, (int)opts.size(), opts.data());
  out->compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  size_t n = 0;
  R.log_size(prog, &n);
  std::string log(n + 1, '\0');
  if (n) R.log(prog, &log[0]);
  if (r != HIPRTC_SUCCESS) {
    R.destroy(&prog);
    char buf[2300];
    snprintf(buf, sizeof buf, "hipRTC compile of the specialised kernels failed: %s\n%.2000s", R.err(r), log.c_str());
    *err = buf;
    return RT_ERR_DEVICE;
  }
  n = 0;
  R.code_size(prog, &n);
  out->code.resize(n);
  R.code(prog, out->code.data());
  R.destroy(&prog);
  code_resources(out);
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

int spec_guard(const SpecCode& c, const std::string& text, std::string* err) {
  const bool def = c.name.rfind("rt_spec_def_", 0) == 0;
  const bool tree = text.find("rows_body<" + std::to_string(RT_MODE_TREE) + ",") != std::string::npos;
  const int max_scratch = def ? RT_SPEC_MAX_SCRATCH_DEF : tree ? RT_SPEC_MAX_SCRATCH_TREE : RT_SPEC_MAX_SCRATCH_ROWS;
  if (c.name.empty() || c.vgprs < 0 || c.scratch < 0) {
    *err = "resource guard: the code object's metadata holds no resource usage for the kernel";
    return RT_ERR_UNSUPPORTED;
  }
  if (c.vgprs > RT_SPEC_MAX_VGPRS || c.scratch > max_scratch) {
    char buf[256];
    snprintf(buf, sizeof buf, "resource guard: %s uses %d VGPRs and %d B/lane of scratch (bounds %d / %d)", c.name.c_str(),
             c.vgprs, c.scratch, RT_SPEC_MAX_VGPRS, max_scratch);
    *err = buf;
    return RT_ERR_UNSUPPORTED;
  }
  return RT_OK;
}

// On-disk cache entry: "RTSPEC03\n", then length-prefixed (u64) identity (spec_build_identity), program
// text, kernel name and code object.  A hit must match identity AND text; the resource numbers the guard
// checks are read from the code object itself (code_resources), never from the file.
void put_blob(std::string& f, const void* p, uint64_t n) {
  f.append((const char*)&n, 8);
  f.append((const char*)p, n);
}
bool get_blob(const std::vector<char>& f, size_t* at, std::string* s) {
  uint64_t n = 0;
  if (*at + 8 > f.size()) return false;
  memcpy(&n, f.data() + *at, 8);
  *at += 8;
  if (n > f.size() - *at) return false;
  s->assign(f.data() + *at, n);
  *at += n;
  return true;
}
std::string disk_path(const std::string& dir, const std::string& identity, const std::string& text) {
  char buf[64];
  snprintf(buf, sizeof buf, "/spec_%016llx.rtco", (unsigned long long)fnv1a(identity + '\0' + text));
  return dir + buf;
}
bool disk_read(const std::string& path, const std::string& identity, const std::string& text, SpecCode* out) {
  FILE* fi = fopen(path.c_str(), "rb");
  if (!fi) return false;
  std::vector<char> f;
  char buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, fi)) > 0) f.insert(f.end(), buf, buf + n);
  fclose(fi);
  static const char magic[] = "RTSPEC03\n";
  if (f.size() < 9 || memcmp(f.data(), magic, 9) != 0) return false;
  size_t at = 9;
  std::string id, tx, name, code;
  if (!get_blob(f, &at, &id) || id != identity || !get_blob(f, &at, &tx) || tx != text || !get_blob(f, &at, &name) ||
      !get_blob(f, &at, &code) || at != f.size())
    return false;
  out->code.assign(code.begin(), code.end());
  code_resources(out);                                    // name and resources from the code object's metadata
  if (out->name != name) return false;
  out->compile_ms = 0.0;
  out->from_disk = true;
  return true;
}
void disk_write(const std::string& dir, const std::string& path, const std::string& identity, const std::string& text,
                const SpecCode& c) {
  for (size_t i = 1; i <= dir.size(); ++i)              // mkdir -p
    if (i == dir.size() || dir[i] == '/') (void)mkdir(dir.substr(0, i).c_str(), 0755);
  std::string f("RTSPEC03\n");
  put_blob(f, identity.data(), identity.size());
  put_blob(f, text.data(), text.size());
  put_blob(f, c.name.data(), c.name.size());
  put_blob(f, c.code.data(), c.code.size());
  char tmp[64];
  snprintf(tmp, sizeof tmp, ".tmp.%d.%llx", (int)getpid(), (unsigned long long)std::hash<std::thread::id>()(std::this_thread::get_id()));
  const std::string tp = path + tmp;
  FILE* fo = fopen(tp.c_str(), "wb");
  if (!fo) return;                                        // the cache is an optimisation: no error
  const bool ok = fwrite(f.data(), 1, f.size(), fo) == f.size();
  if (fclose(fo) == 0 && ok) (void)rename(tp.c_str(), path.c_str());
  else (void)unlink(tp.c_str());
}

// The code object of one program: the on-disk cache, else hipRTC; then the resource guard.
int spec_obtain(const std::string& text, SpecCode* out, std::string* err) {
  const Rtc& R = rtc();
  if (!R.rocm) {
    *err = "hipRTC guard: the ROCm installation's libhiprtc could not be loaded into a namespace of its own (" + R.origin +
           "); another hipRTC in the process (PyTorch bundles an older LLVM) is not used";
    return RT_ERR_UNSUPPORTED;
  }
  std::string dir;
  {
    std::lock_guard<std::mutex> lk(g_spec_mu);
    dir = sst().disk_dir;
  }
  const std::string ident = dir.empty() ? "" : spec_build_identity();
  const std::string path = dir.empty() ? "" : disk_path(dir, ident, text);
  if (!path.empty() && disk_read(path, ident, text, out)) return spec_guard(*out, text, err);
  int rc = spec_compile(text, out, err);
  if (!rc) rc = spec_guard(*out, text, err);
  if (!rc && !path.empty()) disk_write(dir, path, ident, text, *out);
  return rc;
}

void spec_worker() {
  SpecState& S = sst();
  for (;;) {
    std::shared_ptr<SpecJob> j;
    {
      std::unique_lock<std::mutex> lk(g_spec_mu);
      S.qcv.wait(lk, [&] { return S.stop || !S.queue.empty(); });
      if (S.queue.empty()) return;                        // shut down
      j = S.queue.front();
      S.queue.pop_front();
      if (j->interest.load() == 0) {                      // nobody renders this program any more
        auto it = S.jobs.find(j->text);
        if (it != S.jobs.end() && it->second == j) S.jobs.erase(it);
        job_finish(j.get(), SPEC_CANCELLED);
        continue;
      }
      j->state = SPEC_RUNNING;
    }
    std::string err;
    const int rc = spec_obtain(j->text, &j->code, &err);
    if (rc) j->error = err;
    job_finish(j.get(), rc ? SPEC_FAILED : SPEC_DONE);
  }
}

// A token for the program `text`: the process's job for it (queued, running or done), or a new job
// for the pool.  retry: a FAILED job is compiled again.  *was_done: the code object already existed.
std::shared_ptr<SpecJob> spec_request(const std::string& text, bool retry = false, bool* was_done = nullptr) {
  std::lock_guard<std::mutex> lk(g_spec_mu);
  SpecState& S = sst();
  auto it = S.jobs.find(text);
  if (it != S.jobs.end()) {
    const std::shared_ptr<SpecJob> j = it->second;
    const int st = j->state.load();
    if (st != SPEC_CANCELLED && !(retry && st == SPEC_FAILED)) {
      j->last_use = ++S.clock;
      if (was_done) *was_done = st == SPEC_DONE;
      return job_token(j);
    }
    S.jobs.erase(it);
  }
  if (was_done) *was_done = false;
  auto j = std::make_shared<SpecJob>();
  j->text = text;
  j->last_use = ++S.clock;
  if (S.jobs.size() >= RT_SPEC_CACHE_JOBS) {              // evict the least recently used finished jobs nobody holds
    std::vector<std::pair<uint64_t, std::string>> idle;
    for (auto& kv : S.jobs)
      if (kv.second->interest.load() == 0 && job_finished(kv.second.get())) idle.push_back({kv.second->last_use, kv.first});
    std::sort(idle.begin(), idle.end());
    for (size_t i = 0; i < idle.size() && S.jobs.size() >= RT_SPEC_CACHE_JOBS; ++i) S.jobs.erase(idle[i].second);
  }
  S.jobs.emplace(text, j);
  if (S.stop) {
    j->error = "the specialisation pool is shut down (rt_spec_shutdown)";
    j->state = SPEC_FAILED;
    return job_token(j);
  }
  S.queue.push_back(j);
  const size_t want = std::min<size_t>(RT_SPEC_WORKERS_MAX, std::max(1u, std::thread::hardware_concurrency()));
  if (S.workers.size() < want) {
    // A host that exits while a compile runs would tear down hipRTC / LLVM under a live worker: the
    // first worker registers rt_spec_shutdown at exit (it waits for running compiles, cancels queued
    // ones), so every host is covered, not only the Python wrapper (which also calls it).
    static std::once_flag at_exit;
    std::call_once(at_exit, [] { atexit(rt_spec_shutdown); });
    S.workers.emplace_back(spec_worker);
  }
  S.qcv.notify_one();
  return job_token(j);
}

}  // namespace

namespace rt {

const char* spec_compiler() { return rtc().origin.c_str(); }

// The flags of an uploaded scene that decide its program (cheap; no text is generated).
void spec_flags(const FlatScene& f, rt_ctx* c) {
  // The walks unroll over every hierarchy node and leaf, twice (nearest hit, shadows), and the
  // shading over every object: code size and compile time grow with the scene (globes.scene, 6
  // objects and 11 leaves: ~15 k instructions, ~3-12 s of hipRTC per kernel).  Larger scenes keep the
  // generic kernels (fractal.scene: 171 objects).
  c->spec_fits = f.objects.size() <= RT_SPEC_MAX_OBJECTS && f.leaves.size() <= RT_SPEC_MAX_LEAVES;
  c->spec_mode = !f.any_transparent ? RT_MODE_REFL : f.ray_chains ? RT_MODE_CHAIN : RT_MODE_TREE;
  c->spec_fc = f.colour_fast != 0;
  c->spec_deferred = c->spec_mode == RT_MODE_REFL;
}

// The program text of a flattened scene for c's level: a registered family's, or its own.
static void spec_text(const FlatScene& f, rt_ctx* c) {
  spec_flags(f, c);
  c->spec_family = 0;
  {
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

void spec_drop(rt_ctx* c) {
  for (auto& m : c->spec_mods)
    if (m) (void)hipModuleUnload(m);
  memset(c->spec_mods, 0, sizeof c->spec_mods);
  c->spec_mod = nullptr;
  memset(c->spec_rows, 0, sizeof c->spec_rows);
  memset(c->spec_def, 0, sizeof c->spec_def);
  memset(c->spec_prim, 0, sizeof c->spec_prim);
  c->spec_jobs.clear();                                   // drops this context's interest
  c->spec_error.clear();
}

void spec_prepare(rt_ctx* c, bool retry) {
  c->spec_jobs.clear();
  c->spec_error.clear();
  c->spec_note.clear();
  if (!c->spec_on || !c->spec_flat || !c->spec_fits) return;
  spec_text(*c->spec_flat, c);
  bool all_done = true;
  for (const std::string& t : spec_programs(c)) {
    bool done = false;
    c->spec_jobs.push_back(spec_request(t, retry, &done));
    all_done = all_done && done;
  }
  if (all_done) c->spec_note = " [process cache]";
  c->spec_t0 = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int spec_poll(rt_ctx* c) {
  if (c->spec_jobs.empty()) return RT_OK;
  for (auto& j : c->spec_jobs)
    if (!job_finished(j.get())) return RT_PENDING;
  for (auto& j : c->spec_jobs)
    if (j->state.load() != SPEC_DONE) {
      c->spec_error = j->state.load() == SPEC_CANCELLED ? "compile cancelled (rt_spec_shutdown)" : j->error;
      c->spec_jobs.clear();
      return RT_OK;
    }
  char name[32];
  const std::vector<SpecKernel> ks = spec_kernels(c);
  double ms = 0.0;
  bool disk = false;
  std::string res;
  for (size_t i = 0; i < ks.size(); ++i) {
    const SpecKernel& k = ks[i];
    const SpecCode& code = c->spec_jobs[i]->code;
    hipError_t e = hipModuleLoadData(&c->spec_mods[i], code.code.data());
    if (e == hipSuccess) {
      snprintf(name, sizeof name, spec_kernel_name(k.kind), k.f64, k.cal);
      hipFunction_t* fn = k.kind == 2 ? &c->spec_prim[k.f64][k.cal] : k.kind ? &c->spec_def[k.f64][k.cal] : &c->spec_rows[k.f64][k.cal];
      e = hipModuleGetFunction(fn, c->spec_mods[i], name);
    }
    if (e != hipSuccess) {
      c->spec_jobs.clear();
      spec_drop(c);
      c->spec_error = std::string("loading the specialised code object failed: ") + hipGetErrorString(e);
      return RT_OK;
    }
    ms = std::max(ms, code.compile_ms);
    disk = disk || code.from_disk;
    if (i == 0) {
      char b[160];
      snprintf(b, sizeof b, "%d VGPRs (%d spilled), %d B/lane scratch", code.vgprs, code.vspill, code.scratch);
      res = b;
    }
  }
  c->spec_mod = c->spec_mods[0];
  c->spec_hash = fnv1a(c->spec_src);
  c->spec_compile_ms = ms;
  c->spec_res = res;
  if (disk && c->spec_note.empty()) c->spec_note = " [disk cache]";
  c->spec_ready_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count() -
                     c->spec_t0;
  c->spec_jobs.clear();
  // Orders built while the generic kernels ran may have chosen the deferred kernel for a tail-bound
  // launch (split entries); with the specialised megakernel loaded that choice no longer pays
  // (k_rows.hip): those geometries calibrate again.
  for (auto& s : c->order)
    if (s.valid && s.deferred) drop_order(s);
  return RT_OK;
}

int spec_wait(rt_ctx* c, double timeout_ms) {
  const auto t0 = std::chrono::steady_clock::now();
  for (auto& j : c->spec_jobs) {
    double left = -1.0;
    if (timeout_ms >= 0)
      left = std::max(0.0, timeout_ms - std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    if (!job_wait(j.get(), left)) return RT_PENDING;
  }
  return spec_poll(c);
}

}  // namespace rt

// Waits for every job (no limit); the longest fresh compile in *ms (0: all came from a cache); the
// first failure's status and message.
static int wait_all(const std::vector<std::shared_ptr<SpecJob>>& jobs, const std::vector<bool>& was_done, double* ms) {
  *ms = 0.0;
  for (size_t i = 0; i < jobs.size(); ++i) {
    job_wait(jobs[i].get(), -1.0);
    if (jobs[i]->state.load() != SPEC_DONE)
      return fail(RT_ERR_UNSUPPORTED, "%s", jobs[i]->state.load() == SPEC_CANCELLED ? "compile cancelled (rt_spec_shutdown)"
                                                                                   : jobs[i]->error.c_str());
    if (!was_done[i]) *ms = std::max(*ms, jobs[i]->code.compile_ms);
  }
  return RT_OK;
}

// The programs of scene s at level `level` (tmp context), requested from the pool.
static int scene_jobs(const rt_scene* s, int level, rt_ctx* tmp, std::vector<std::shared_ptr<SpecJob>>* jobs,
                      std::vector<bool>* was_done) {
  if (!s) return fail(RT_ERR_INVALID, "null scene");
  rt::FlatScene f;
  int rc = rt::flatten(*s, &f);
  if (rc) return rc;
  tmp->spec_on = level;
  rt::spec_text(f, tmp);
  if (!tmp->spec_fits)
    return fail(RT_ERR_UNSUPPORTED, "scene of %zu objects / %zu leaves is not specialised (limits %d / %d)",
                f.objects.size(), f.leaves.size(), RT_SPEC_MAX_OBJECTS, RT_SPEC_MAX_LEAVES);
  for (const std::string& t : rt::spec_programs(tmp)) {
    bool done = false;
    jobs->push_back(spec_request(t, false, &done));
    was_done->push_back(done);
  }
  return RT_OK;
}

// rt_scene_precompile (include/rt_abi.h): the specialised programs of a scene into the process cache,
// no device needed -- a host may compile on a worker thread while it renders with the generic kernels
extern "C" int rt_scene_precompile(const rt_scene* s, double* compile_ms) {
  rt_ctx tmp;
  std::vector<std::shared_ptr<SpecJob>> jobs;
  std::vector<bool> done;
  double ms = 0.0;
  int rc = scene_jobs(s, 1, &tmp, &jobs, &done);
  if (!rc) rc = wait_all(jobs, done, &ms);
  if (compile_ms) *compile_ms = ms;
  return rc;
}

// rt_scene_spec_report (include/rt_abi.h): compile (or find) the scene's level-1 programs and describe
// them: the compiler, and per kernel its resource use and how it was obtained
extern "C" int rt_scene_spec_report(const rt_scene* s, char* buf, size_t cap, size_t* len) {
  if (!len || (cap > 0 && !buf)) return fail(RT_ERR_INVALID, "null argument");
  rt_ctx tmp;
  std::vector<std::shared_ptr<SpecJob>> jobs;
  std::vector<bool> done;
  double ms = 0.0;
  int rc = scene_jobs(s, 1, &tmp, &jobs, &done);
  if (!rc) rc = wait_all(jobs, done, &ms);
  if (rc) return rc;
  // source: how the code object was made -- by hipRTC in this process, or read from the disk cache
  std::string text = "compiler: " + rtc().identity + (rtc().rocm ? " (the ROCm installation's hipRTC)" : "") + "\n";
  for (size_t i = 0; i < jobs.size(); ++i) {
    const SpecCode& c = jobs[i]->code;
    char line[512];
    snprintf(line, sizeof line, "%s: vgprs %d spilled %d sgprs %d scratch %d occupancy %d code %zu compile_ms %.0f source %s\n",
             c.name.c_str(), c.vgprs, c.vspill, c.sgprs, c.scratch, c.occupancy, c.code.size(), c.compile_ms,
             c.from_disk ? "disk" : "hiprtc");
    text += line;
  }
  *len = text.size();
  if (cap > 0) {
    const size_t n = text.size() < cap - 1 ? text.size() : cap - 1;
    memcpy(buf, text.data(), n);
    buf[n] = 0;
  }
  return RT_OK;
}

// rt_scene_spec_program (include/rt_abi.h): the prelude and every kernel rt_scene_precompile compiles
extern "C" int rt_scene_spec_program(const rt_scene* s, char* buf, size_t cap, size_t* len) {
  if (!s || !len || (cap > 0 && !buf)) return fail(RT_ERR_INVALID, "null argument");
  rt::FlatScene f;
  int rc = rt::flatten(*s, &f);
  if (rc) return rc;
  rt_ctx tmp;
  tmp.spec_on = 2;
  rt::spec_text(f, &tmp);
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
// contexts whose scene belongs to a class load its program (spec_text).
static bool same_hierarchy(const std::vector<RtTrav>& a, const std::vector<RtTrav>& b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (a[i].obj != b[i].obj || a[i].skip != b[i].skip) return false;
  return true;
}
extern "C" int rt_spec_family_register(const rt_scene* const* scenes, int32_t n, double* compile_ms) {
  if (compile_ms) *compile_ms = 0.0;
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
      if (fams.size() >= RT_SPEC_MAX_FAMILIES)             // every family is a compile: bounded per call
        return fail(RT_ERR_UNSUPPORTED, "the scenes form more than %d families (structure or object hierarchy differ)",
                    RT_SPEC_MAX_FAMILIES);
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
  // A family of ONE scene gets no family program: the scene's own program (every word a constant, the
  // tables in the constant address space) is the better code -- globes.scene as a family of one
  // spilled to 1 392 B/lane of scratch (its own program: 560) -- so its own program is compiled now.
  std::vector<std::shared_ptr<SpecJob>> all;
  std::vector<bool> done;
  std::vector<size_t> first(fams.size());
  for (size_t fi = 0; fi < fams.size(); ++fi) {
    auto& F = fams[fi];
    rt_ctx tmp;
    tmp.spec_on = 1;
    rt::spec_flags(F->base, &tmp);                 // mode / clamp form / size limits of the class
    if (!tmp.spec_fits)
      return fail(RT_ERR_UNSUPPORTED, "scenes of %zu objects / %zu leaves are not specialised (limits %d / %d)",
                  F->base.objects.size(), F->base.leaves.size(), RT_SPEC_MAX_OBJECTS, RT_SPEC_MAX_LEAVES);
    F->src = rt::spec_source(F->base, F->members > 1 ? F.get() : nullptr);
    tmp.spec_src = F->src;
    first[fi] = all.size();
    for (const std::string& t : rt::spec_programs(&tmp)) {
      bool d = false;
      F->jobs.push_back(spec_request(t, false, &d));
      all.push_back(F->jobs.back());
      done.push_back(d);
    }
  }
  // every class's programs, compiled by the pool in parallel; the families whose programs compiled and
  // passed the guard are registered, the others not (their scenes then compile their own programs)
  double ms = 0.0;
  std::string first_err;
  std::vector<char> good(fams.size(), 0);
  for (size_t fi = 0; fi < fams.size(); ++fi) {
    bool ok = true;
    for (size_t i = first[fi]; i < first[fi] + fams[fi]->jobs.size(); ++i) {
      job_wait(all[i].get(), -1.0);
      if (all[i]->state.load() != SPEC_DONE) {
        ok = false;
        if (first_err.empty())
          first_err = "family of " + std::to_string(fams[fi]->members) + " scenes: " +
                      (all[i]->state.load() == SPEC_CANCELLED ? std::string("compile cancelled (rt_spec_shutdown)") : all[i]->error);
      } else if (!done[i]) {
        ms = std::max(ms, all[i]->code.compile_ms);
      }
    }
    good[fi] = ok;
  }
  {
    std::lock_guard<std::mutex> lk(g_spec_mu);
    for (size_t fi = 0; fi < fams.size(); ++fi)
      if (good[fi]) (fams[fi]->members > 1 ? g_families : g_singles).push_back(fams[fi]);   // singles: their own program resident
  }
  if (compile_ms) *compile_ms = ms;
  if (!first_err.empty()) return fail(RT_ERR_UNSUPPORTED, "%s", first_err.c_str());
  return RT_OK;
}

// rt_spec_family_clear (include/rt_abi.h): forget every registered family (loaded modules stay)
extern "C" int rt_spec_family_clear(void) {
  std::vector<std::shared_ptr<SpecFamily>> old, old1;
  {
    std::lock_guard<std::mutex> lk(g_spec_mu);
    old.swap(g_families);
    old1.swap(g_singles);
  }
  return RT_OK;                                    // `old` drops the families' interest in their programs
}

// rt_spec_cache_dir (include/rt_abi.h): the on-disk code-object cache ("" or NULL: none)
extern "C" int rt_spec_cache_dir(const char* dir) {
  std::lock_guard<std::mutex> lk(g_spec_mu);
  sst().disk_dir = dir ? dir : "";
  while (sst().disk_dir.size() > 1 && sst().disk_dir.back() == '/') sst().disk_dir.pop_back();
  return RT_OK;
}

// rt_spec_compiler_info (include/rt_abi.h): which hipRTC the programs compile with
extern "C" int rt_spec_compiler_info(char* buf, size_t cap, int32_t* rocm) {
  const Rtc& R = rtc();
  if (rocm) *rocm = R.rocm ? 1 : 0;
  if (buf && cap > 0) snprintf(buf, cap, "%s", spec_build_identity().c_str());
  return RT_OK;
}

// rt_spec_shutdown (include/rt_abi.h): cancel queued compiles, wait for running ones, stop the pool
extern "C" void rt_spec_shutdown(void) {
  std::vector<std::thread> th;
  {
    std::lock_guard<std::mutex> lk(g_spec_mu);
    SpecState& S = sst();
    S.stop = true;
    for (auto& j : S.queue) {
      auto it = S.jobs.find(j->text);
      if (it != S.jobs.end() && it->second == j) S.jobs.erase(it);
      job_finish(j.get(), SPEC_CANCELLED);
    }
    S.queue.clear();
    th.swap(S.workers);
    S.qcv.notify_all();
  }
  for (auto& t : th) t.join();
}
