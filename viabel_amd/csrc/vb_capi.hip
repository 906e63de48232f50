// vb_capi.hip — the extern "C" boundary declared in include/viabel_amd.h.
//
// Host-side responsibilities: argument validation with the reference's error
// conditions, host/device pointer detection + staging, device-resident
// optimiser state (vb_run), chunked launches, thread-local error strings.
#include "../../include/viabel_amd.h"
#include "vb_internal.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <set>
#include <string>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define VB_HIP(expr)                                                                  \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess)                                                             \
      return fail(VB_EDEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                  __FILE__, __LINE__);                                                \
  } while (0)

#define VB_TRY(expr)             \
  do {                           \
    int rc_ = (expr);            \
    if (rc_ != VB_OK) return rc_; \
  } while (0)

// 0: host memory (staged through the context's buffers); 1: device memory the
// context's GPU can use in place; -1: device memory of another GPU (rejected:
// the kernels would read or write it across devices).  Entry points select the
// context's device first (check_ctx), so hipGetDevice names it.
int ptr_class(const void* p) {
  if (!p) return 0;
  hipPointerAttribute_t at;
  hipError_t e = hipPointerGetAttributes(&at, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  if (at.type == hipMemoryTypeManaged || at.type == hipMemoryTypeUnified) return 1;
  if (at.type != hipMemoryTypeDevice) return 0;
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) return 1;
  return at.device == cur ? 1 : -1;
}

bool is_device_ptr(const void* p) { return ptr_class(p) == 1; }

int foreign_ptr_error(const void* p) {
  hipPointerAttribute_t at;
  int cur = -1;
  (void)hipPointerGetAttributes(&at, p);
  (void)hipGetDevice(&cur);
  return fail(VB_EINVAL, "device pointer %p is on GPU %d but the context is on GPU %d", p,
              at.device, cur);
}

// Device blocks of runs and contexts are cached by (device, size class) instead of
// going back to hipFree: a run made and dropped per call (adagrad_optimize, the
// restart table) paid one hipFree per buffer -- each one synchronises the device and
// unmaps the block, ~0.8 ms for config 5's run -- and a hipMalloc per buffer on the
// next call.  A block is returned only when no work can still use it (vb_run_destroy
// and vb_ctx_destroy synchronise their streams first; a buffer that grows
// synchronises the device before handing its old block back, as hipFree did).  The
// cache is trimmed (hipFree of every cached block) when a hipMalloc fails, and at
// exit by release_live_contexts, before the HIP runtime's own teardown; blocks
// returned after that are freed directly.
namespace devpool {
std::mutex mu;
std::multimap<std::pair<int, size_t>, void*>* cached = nullptr;   // never freed
size_t cached_bytes = 0;
bool closed = false;
// blocks beyond this much cached memory are freed when returned (other allocators,
// torch's among them, share the device's HBM and cannot empty this cache)
constexpr size_t kCacheMax = size_t(8) << 30;

// size class: powers of two up to 4 MB (at least 4 KB), then multiples of 2 MB
size_t size_class(size_t b) {
  if (b <= 4096) return 4096;
  if (b <= (size_t(4) << 20)) {
    size_t c = 8192;
    while (c < b) c <<= 1;
    return c;
  }
  const size_t g = size_t(2) << 20;
  return (b + g - 1) / g * g;
}

void trim_locked() {
  if (!cached) return;
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (auto& kv : *cached) {
    (void)hipSetDevice(kv.first.first);
    (void)hipFree(kv.second);
  }
  cached->clear();
  cached_bytes = 0;
  (void)hipSetDevice(cur);
}

void trim() {
  std::lock_guard<std::mutex> lk(mu);
  trim_locked();
}

// exit: free every cached block; later returns go straight to hipFree
void close() {
  std::lock_guard<std::mutex> lk(mu);
  trim_locked();
  closed = true;
}

hipError_t alloc(void** p, size_t bytes, size_t* cap, int* dev) {
  (void)hipGetDevice(dev);
  const size_t cls = size_class(bytes);
  {
    std::lock_guard<std::mutex> lk(mu);
    if (cached) {
      auto it = cached->find({*dev, cls});
      if (it != cached->end()) {
        *p = it->second;
        cached->erase(it);
        cached_bytes -= cls;
        *cap = cls;
        return hipSuccess;
      }
    }
  }
  hipError_t e = hipMalloc(p, cls);
  if (e != hipSuccess) {   // blocks of other sizes may be what is missing
    (void)hipGetLastError();
    trim();
    e = hipMalloc(p, cls);
  }
  if (e == hipSuccess) *cap = cls;
  return e;
}

void give_back(void* p, size_t cap, int dev) {
  std::lock_guard<std::mutex> lk(mu);
  if (closed || cached_bytes + cap > kCacheMax) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(dev);
    (void)hipFree(p);
    (void)hipSetDevice(cur);
    return;
  }
  if (!cached) cached = new std::multimap<std::pair<int, size_t>, void*>();
  cached->insert({{dev, cap}, p});
  cached_bytes += cap;
}
}  // namespace devpool

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int dev = 0;
  int reserve(size_t bytes) {
    if (bytes <= cap) return VB_OK;
    if (p) {
      (void)hipDeviceSynchronize();   // work queued on the old block finishes first
      devpool::give_back(p, cap, dev);
    }
    p = nullptr;
    cap = 0;
    if (bytes == 0) return VB_OK;
    hipError_t e = devpool::alloc(&p, bytes, &cap, &dev);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      p = nullptr;
      cap = 0;
      return fail(VB_ENOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    }
    return VB_OK;
  }
  // (owners synchronise their streams before they drop their buffers)
  ~DevBuf() {
    if (p) devpool::give_back(p, cap, dev);
  }
  double* d() const { return static_cast<double*>(p); }
};

// Pinned host memory (hipHostMalloc), grown on demand, freed with its owner.
struct PinnedBuf {
  void* p = nullptr;
  size_t cap = 0;
  int reserve(size_t bytes) {
    if (bytes <= cap) return VB_OK;
    release();
    hipError_t e = hipHostMalloc(&p, bytes);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      p = nullptr;
      return fail(VB_ENOMEM, "hipHostMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    }
    cap = bytes;
    return VB_OK;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  ~PinnedBuf() { release(); }
};

}  // namespace

int vbk::vb_set_error(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

struct vb_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  DevBuf slot[16];
  vbk::FrWork* fr = nullptr;  // full-rank workspace, created on first use
  // pre-draw overlap (predraw_overlap_streams): two streams on disjoint CU halves
  // and the events that chain them; created on first use, -1 not tried, 0 failed
  int pd_ready = -1;
  hipStream_t pd_stream = nullptr, blk_stream = nullptr;
  hipEvent_t pd_ev[6] = {};
  PinnedBuf psis_flags;  // the PSIS fast select's per-column flags, read by the host
  // progress snapshots (vb_run_values_async): one pinned buffer per context, reused by
  // its runs (a hipHostMalloc per run cost ~0.3 ms per adagrad_optimize call); the
  // run whose snapshot it holds, and that snapshot's event
  PinnedBuf vals_pin;
  const void* vals_owner = nullptr;
  hipEvent_t vals_ev = nullptr;
  // the resources the context created besides its stream: the full-rank workspace
  // (rocBLAS / rocSOLVER handles, buffers), the CU-masked pre-draw streams and their
  // events.  Run by vb_ctx_destroy and, for contexts still alive at exit, by the
  // library's own exit handler (release_live_contexts) before the HIP runtime tears
  // itself down.  Idempotent; the context stays usable (they are made again on use).
  void release_side() {
    if (pd_stream) (void)hipStreamSynchronize(pd_stream);
    if (blk_stream) (void)hipStreamSynchronize(blk_stream);
    vbk::fr_work_destroy(fr);
    fr = nullptr;
    for (hipEvent_t& e : pd_ev) {
      if (e) (void)hipEventDestroy(e);
      e = nullptr;
    }
    if (pd_stream) (void)hipStreamDestroy(pd_stream);
    if (blk_stream) (void)hipStreamDestroy(blk_stream);
    pd_stream = blk_stream = nullptr;
    pd_ready = -1;
    psis_flags.release();
    if (vals_ev) (void)hipEventSynchronize(vals_ev);
    vals_pin.release();
    vals_owner = nullptr;
    if (vals_ev) (void)hipEventDestroy(vals_ev);
    vals_ev = nullptr;
  }
  ~vb_ctx() { release_side(); }
};

namespace {

// Contexts alive now.  A process that exits with contexts it never destroyed (a
// Python program whose objects are still referenced, a C program without
// vb_ctx_destroy) would otherwise leave their CU-masked streams and rocBLAS
// handles to the process's static teardown, after the HIP runtime's: under
// rocprofv3 that order crashed at exit (round 5).  The handler is registered with
// std::atexit after the first context exists, i.e. after the HIP runtime has
// initialised, so it runs before the runtime's own exit-time teardown.
std::mutex g_ctx_mu;
std::set<vb_ctx*>* g_live = nullptr;

void release_live_contexts() {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  if (!g_live) return;
  for (vb_ctx* c : *g_live) {
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    c->release_side();
  }
  // every cached device block (runs and contexts still alive free theirs directly)
  devpool::close();
}

void register_ctx(vb_ctx* c) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  if (!g_live) {
    g_live = new std::set<vb_ctx*>();  // never freed: read by the exit handler
    std::atexit(release_live_contexts);
  }
  g_live->insert(c);
}

void unregister_ctx(vb_ctx* c) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  if (g_live) g_live->erase(c);
}

}  // namespace

namespace {

// An input argument: device pointer used directly, host pointer staged.
struct In {
  const double* d = nullptr;
  int stage(vb_ctx* c, int s, const double* p, size_t count) {
    if (!p || count == 0) {
      d = p;
      return VB_OK;
    }
    const int pc = ptr_class(p);
    if (pc < 0) return foreign_ptr_error(p);
    if (pc == 1) {
      d = p;
      return VB_OK;
    }
    VB_TRY(c->slot[s].reserve(count * sizeof(double)));
    VB_HIP(hipMemcpyAsync(c->slot[s].p, p, count * sizeof(double), hipMemcpyHostToDevice,
                          c->stream));
    d = c->slot[s].d();
    return VB_OK;
  }
};

// An output argument: device pointer written directly, host pointer copied back.
template <class T>
struct OutT {
  T* user = nullptr;
  T* d = nullptr;
  size_t count = 0;
  bool host = false;
  int stage(vb_ctx* c, int s, T* p, size_t n) {
    user = p;
    count = n;
    if (!p || n == 0) {
      d = p;
      return VB_OK;
    }
    const int pc = ptr_class(p);
    if (pc < 0) return foreign_ptr_error(p);
    if (pc == 1) {
      d = p;
      return VB_OK;
    }
    host = true;
    VB_TRY(c->slot[s].reserve(n * sizeof(T)));
    d = static_cast<T*>(c->slot[s].p);
    return VB_OK;
  }
  int finish(vb_ctx* c) {
    if (host && count)
      VB_HIP(hipMemcpyAsync(user, d, count * sizeof(T), hipMemcpyDeviceToHost, c->stream));
    return VB_OK;
  }
};
using Out = OutT<double>;

int sync(vb_ctx* c) {
  VB_HIP(hipStreamSynchronize(c->stream));
  return VB_OK;
}

// Block-kernel work with Philox draws of the mean-field t family always
// pre-draws them (launch_block_predraw + the device-noise path: the t draws are a
// step's critical path); the Gaussian family draws in kernel unless
// VIABEL_AMD_PREDRAW=all (read per call: tests switch it).  Chunks hold at most
// kPredrawBytes of draws and kPredrawMaxSteps steps.
constexpr size_t kPredrawBytes = size_t(256) << 20;
constexpr long long kPredrawMaxSteps = 512;
constexpr long long kPredrawOverlapMinProblems = 8;   // overlapped pre-draw (below)
int block_pf_enabled();

// VIABEL_AMD_HOST_TRACE=1: per-call host timestamps of a launch path to stderr
// (measurement only; one getenv per process)
struct HostTrace {
  static bool on() {
    static const bool v = [] {
      const char* e = std::getenv("VIABEL_AMD_HOST_TRACE");
      return e && e[0] == '1';
    }();
    return v;
  }
  std::chrono::steady_clock::time_point t[8];
  int n = 0;
  HostTrace() {
    if (on()) t[n++] = std::chrono::steady_clock::now();
  }
  void mark() {
    if (on() && n < 8) t[n++] = std::chrono::steady_clock::now();
  }
  void print(const char* what) const {
    if (!on()) return;
    std::fprintf(stderr, "[host] %s:", what);
    for (int i = 1; i < n; ++i)
      std::fprintf(stderr, " %.2f", std::chrono::duration<double, std::micro>(t[i] - t[i - 1]).count());
    std::fprintf(stderr, " us\n");
  }
};
// VIABEL_AMD_PREDRAW: unset -> the t family pre-draws, and the Gaussian family in
// optimisation runs whose rows the block kernel's copy wave stages (block_pf_layout);
// "t" -> the t family only; "all" -> every family and call; "0" -> in-kernel draws
// for every family (same bits either way)
bool predraw_enabled(int fam_kind, bool run = false, int N = 0, int D = 0, bool need_lq = false) {
  const char* e = std::getenv("VIABEL_AMD_PREDRAW");
  if (e && e[0] == '0') return false;
  if (fam_kind == VB_FAMILY_MF_T) return true;
  if (e && e[0] == 'a') return true;
  if (e && e[0] == 't') return false;
  return run && block_pf_enabled() && vbk::block_pf_layout(N, D, need_lq, block_pf_enabled());
}

// VIABEL_AMD_FR_FUSE=0: the full-rank step keeps its separate unpack / power /
// draw / rows / colsum / pack / adagrad launches (A/B switch; same results to
// rounding)
bool fr_fuse_enabled() {
  const char* e = std::getenv("VIABEL_AMD_FR_FUSE");
  return !(e && e[0] == '0');
}

// VIABEL_AMD_BLOCK_PF=0: the block kernel's device-noise rows are read straight
// from HBM by the row threads instead of staged into LDS by a copy wave (A/B
// switch; same bits)
// VIABEL_AMD_BLOCK_SPLIT=0: the copy-wave layout keeps one row thread per sample
// instead of two (each lane of a pair takes half of the sample's coordinates,
// block_layout); the value is the BlockArgs::pf mode: 0 off, 1 copy wave, 2 copy
// wave with split rows where the layout allows them
int block_pf_enabled() {
  static const int on = [] {
    const char* e = std::getenv("VIABEL_AMD_BLOCK_PF");
    if (e && e[0] == '0') return 0;
    const char* sp = std::getenv("VIABEL_AMD_BLOCK_SPLIT");
    return (sp && sp[0] == '0') ? 1 : 2;
  }();
  return on;
}

// VIABEL_AMD_PREDRAW_OVERLAP=0: the pre-draw of chunk k + 1 waits for the block
// kernel of chunk k (one stream) instead of running beside it on the other half of
// the CUs (predraw_overlap_streams)
bool predraw_overlap_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("VIABEL_AMD_PREDRAW_OVERLAP");
    return !(e && e[0] == '0');
  }();
  return on;
}

int check_ctx(vb_ctx* c) {
  if (!c) return fail(VB_EINVAL, "null vb_ctx");
  VB_HIP(hipSetDevice(c->device));
  return VB_OK;
}

// The overlapped pre-draw's streams: the block kernel's latency-bound workgroups
// (one per problem) on the even CUs, the throughput pre-draw of the next chunk on
// the odd CUs (hipExtStreamCreateWithCUMask), so that neither shares a CU with the
// other (a pre-draw beside the block kernel on shared CUs slowed the fit 18.7 ->
// 26.5 ms).  Returns false (serial pre-draw) if the masks are refused.
bool predraw_overlap_streams(vb_ctx* c) {
  if (c->pd_ready >= 0) return c->pd_ready == 1;
  c->pd_ready = 0;
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess ||
      ncu < 8 || ncu > 1024) {
    (void)hipGetLastError();
    return false;
  }
  // the block kernel on the first half of the CU ids, the pre-draw on the second
  // (measured against even / odd ids and an unmasked block stream: config 5's fit
  // 14.8-14.9 / 15.0-15.3 / 15.2-15.3 ms, profiles/r04/predraw_mask_ab.log)
  std::vector<uint32_t> first((ncu + 31) / 32, 0u), second((ncu + 31) / 32, 0u);
  for (int i = 0; i < ncu; ++i) (i >= ncu / 2 ? second : first)[i / 32] |= 1u << (i % 32);
  hipError_t e1 = hipExtStreamCreateWithCUMask(&c->blk_stream, (uint32_t)first.size(), first.data());
  if (e1 != hipSuccess ||
      hipExtStreamCreateWithCUMask(&c->pd_stream, (uint32_t)second.size(), second.data()) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  for (hipEvent_t& e : c->pd_ev)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
  c->pd_ready = 1;
  return true;
}

struct FamInfo {
  int kind;
  int D;
  size_t P;  // length of lambda
  double df, t_scale, shape, t_const;
};

int check_family(const vb_family* f, FamInfo* o) {
  if (!f) return fail(VB_EINVAL, "null vb_family");
  if (f->kind != VB_FAMILY_MF_GAUSSIAN && f->kind != VB_FAMILY_MF_T && f->kind != VB_FAMILY_FR_T)
    return fail(VB_EUNSUPPORTED, "family kind %d is not implemented on the device", f->kind);
  if (f->dim < 1 || f->dim > (1LL << 30)) return fail(VB_EINVAL, "invalid dimension %lld", (long long)f->dim);
  o->kind = f->kind;
  o->D = (int)f->dim;
  o->P = 2 * (size_t)f->dim;
  o->df = f->df;
  o->t_scale = o->shape = o->t_const = 0.0;
  if (f->kind == VB_FAMILY_FR_T) {
    if (!(f->df > 2)) return fail(VB_EINVAL, "df must be greater than 2");  // vb.py:193-194
    if (f->dim > 8192) return fail(VB_EUNSUPPORTED, "full-rank family needs D <= 8192");
    const double D = (double)f->dim;
    o->P = (size_t)f->dim + (size_t)f->dim * (f->dim + 1) / 2;
    // multivariate_t_logpdf constant (_distributions.py:33-34)
    o->t_const = std::lgamma(0.5 * (f->df + D)) - std::lgamma(0.5 * f->df) -
                 0.5 * D * std::log(M_PI * f->df);
    return VB_OK;
  }
  if (f->kind == VB_FAMILY_MF_T) {
    if (!(f->df > 2)) return fail(VB_EINVAL, "df must be greater than 2");  // vb.py:141-142
    o->t_scale = std::sqrt(f->df / 2.0);
    o->shape = f->df / 2.0;
    // scipy.stats.t._logpdf constant: gammaln((df+1)/2) - gammaln(df/2) - 0.5*log(df*pi)
    o->t_const = std::lgamma(0.5 * (f->df + 1.0)) - std::lgamma(0.5 * f->df) -
                 0.5 * std::log(f->df * M_PI);
  }
  return VB_OK;
}

int check_target(const vb_target* t, int D) {
  if (!t) return fail(VB_EINVAL, "null vb_target");
  if (t->kind < VB_TARGET_ISOGAUSS || t->kind > VB_TARGET_CALLBACK)
    return fail(VB_EUNSUPPORTED, "target kind %d is not implemented on the device", t->kind);
  if (t->kind == VB_TARGET_CALLBACK && !t->callback)
    return fail(VB_EINVAL, "callback target needs a callback");
  if (t->kind == VB_TARGET_CORR_GAUSS &&
      (!t->params || t->n_params != (int64_t)t->dim * t->dim + 1))
    return fail(VB_EINVAL, "corr_gauss target needs D*D + 1 parameters (precision, log normaliser)");
  if (t->dim != D)
    return fail(VB_EINVAL, "target dimension %lld does not match family dimension %d",
                (long long)t->dim, D);
  if (t->kind == VB_TARGET_FUNNEL && D < 2) return fail(VB_EINVAL, "funnel target needs D >= 2");
  if (t->kind == VB_TARGET_EIGHT_SCHOOLS_NCP && D != 10)
    return fail(VB_EINVAL, "eight_schools_ncp target has dimension 10, got %d", D);
  return VB_OK;
}

void key_of(uint64_t seed, uint32_t* k0, uint32_t* k1) {
  *k0 = (uint32_t)(seed & 0xffffffffu);
  *k1 = (uint32_t)(seed >> 32);
}

// Device copy of a target's parameters and its scalar log normaliser.
int target_params(vb_ctx* c, int s, const vb_target* t, const double** dev, double* tconst) {
  *dev = nullptr;
  *tconst = 0.0;
  if (t->kind != VB_TARGET_CORR_GAUSS) return VB_OK;
  const size_t dd = (size_t)t->dim * t->dim;
  In in;
  VB_TRY(in.stage(c, s, t->params, dd + 1));
  *dev = in.d;
  VB_HIP(hipMemcpyAsync(tconst, in.d + dd, sizeof(double), hipMemcpyDeviceToHost, c->stream));
  VB_HIP(hipStreamSynchronize(c->stream));
  return VB_OK;
}

int fr_work(vb_ctx* c, vbk::FrWork** w) {
  if (!c->fr) c->fr = vbk::fr_work_create();
  if (!c->fr) return fail(VB_ENOMEM, "out of host memory");
  *w = c->fr;
  return VB_OK;
}

int require_fr(int fam_kind, int tgt_kind) {
  if (tgt_kind == VB_TARGET_CORR_GAUSS && fam_kind != VB_FAMILY_FR_T)
    return fail(VB_EUNSUPPORTED, "the corr_gauss target is implemented for the full-rank family only");
  return VB_OK;
}

vbk::HostTarget host_of(const vb_target* t) {
  vbk::HostTarget h{};
  if (t && t->kind == VB_TARGET_CALLBACK) {
    h.fn = t->callback;
    h.user = t->user;
  }
  return h;
}

vbk::FrSpec fr_spec(const FamInfo& fi, const vb_target* tgt, const vb_objective* obj,
                    const double* tparams, double tconst) {
  vbk::FrSpec f{};
  f.host = host_of(tgt);
  f.D = fi.D;
  f.N = (int)obj->n_samples;
  f.tgt = tgt->kind;
  f.chivi = obj->kind == VB_OBJ_CHIVI;
  f.pd = obj->kind == VB_OBJ_KLVI_PD;
  f.df = fi.df;
  f.t_const = fi.t_const;
  f.alpha = obj->alpha;
  f.tparams = tparams;
  f.tconst = tconst;
  return f;
}

// Constant of the column-pair kernel's value: KLVI -(c0 + sum log s + mean log p);
// KLVI_PD adds -log q's per-coordinate constants instead (the kernel accumulates
// 1/2 eps^2 or (df+1)/2 log1p(eps^2/df) with log p).
double sep_c0(const FamInfo& fi, bool pd) {
  const double D = (double)fi.D;
  if (fi.kind == VB_FAMILY_MF_T) return pd ? -D * fi.t_const : 0.0;
  return pd ? 0.5 * D * std::log(2 * M_PI) : 0.5 * D * (1.0 + std::log(2 * M_PI));
}

vbk::MfSpec mf_spec(const FamInfo& fi, const vb_target* tgt, const vb_objective* obj) {
  vbk::MfSpec f{};
  f.host = host_of(tgt);
  f.fam = fi.kind;
  f.D = fi.D;
  f.N = obj ? (int)obj->n_samples : 0;
  f.tgt = tgt->kind;
  f.chivi = obj && obj->kind == VB_OBJ_CHIVI;
  f.pd = obj && obj->kind == VB_OBJ_KLVI_PD;
  f.alpha = obj ? obj->alpha : 2.0;
  f.t_scale = fi.t_scale;
  f.shape = fi.shape;
  f.df = fi.df;
  f.t_const = fi.t_const;
  return f;
}

// vb_objective_value_grad for the full-rank t family
int fr_objective(vb_ctx* c, const FamInfo& fi, const vb_target* tgt, const vb_objective* obj,
                 const double* lam, const vb_noise* noise, double* value, double* grad) {
  const bool host = noise->kind == VB_NOISE_HOST;
  if (host && !noise->eps) return fail(VB_EINVAL, "host noise requires eps");
  const size_t N = (size_t)obj->n_samples;
  In dl, dn;
  Out dg;
  VB_TRY(dl.stage(c, 0, lam, fi.P));
  if (host) VB_TRY(dn.stage(c, 1, noise->eps, N * fi.D + N));
  VB_TRY(dg.stage(c, 2, grad, fi.P));
  const double* tp;
  double tc;
  VB_TRY(target_params(c, 3, tgt, &tp, &tc));
  VB_TRY(c->slot[4].reserve(sizeof(double) * 2));
  uint32_t k0, k1;
  key_of(noise->seed, &k0, &k1);
  vbk::FrWork* W;
  VB_TRY(fr_work(c, &W));
  // a root or gradient solve that needed more iterations than launched (an
  // ill-conditioned Sigma) runs the call again with larger counts (fr_info)
  for (int attempt = 0;; ++attempt) {
    VB_TRY(vbk::fr_value_grad(W, fr_spec(fi, tgt, obj, tp, tc), dl.d, host ? dn.d : nullptr, k0,
                              k1, noise->stream, (uint32_t)noise->step, c->slot[4].d(), dg.d,
                              c->stream));
    VB_TRY(sync(c));
    bool again = false;
    if (int rc = vbk::fr_info(W, c->stream, attempt < 16 ? &again : nullptr)) return rc;
    if (!again) break;
  }
  vbk::fr_retry_done(W);
  VB_HIP(hipMemcpyAsync(value, c->slot[4].p, sizeof(double), hipMemcpyDefault, c->stream));
  VB_TRY(dg.finish(c));
  VB_TRY(sync(c));
  return VB_OK;
}

vbk::LrSched make_sched(long long n, double lr, double lr_end) {
  vbk::LrSched s{};
  s.lr = lr;
  s.has_end = !std::isnan(lr_end);
  s.lr_end = s.has_end ? lr_end : 0.0;
  if (s.has_end) {
    // vb.py:332-335, same expression order as the reference
    s.b = ((double)n * lr_end) / (2.0 * (lr - lr_end));
    s.a = lr * s.b;
    s.start = n / 4;
    s.end = (3 * n) / 4;
  }
  return s;
}

}  // namespace

// ===========================================================================
extern "C" {

int vb_abi_version(void) { return VB_ABI_VERSION; }

const char* vb_last_error(void) { return g_err.c_str(); }

#ifndef VB_SRC_HASH
#define VB_SRC_HASH "unknown"
#endif
const char* vb_build_id(void) { return VB_SRC_HASH; }

double vb_flop_tally(int reset) {
  const double t = vbk::gemm_flop_tally();
  if (reset) vbk::gemm_flop_tally() = 0.0;
  return t;
}

int vb_ctx_create(int device, void* hip_stream, vb_ctx** out) {
  if (!out) return fail(VB_EINVAL, "null output pointer");
  *out = nullptr;
  int n = 0;
  VB_HIP(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(VB_EINVAL, "device %d out of range (%d devices)", device, n);
  VB_HIP(hipSetDevice(device));
  vb_ctx* c = new (std::nothrow) vb_ctx();
  if (!c) return fail(VB_ENOMEM, "out of host memory");
  c->device = device;
  if (hip_stream) {
    c->stream = static_cast<hipStream_t>(hip_stream);
  } else {
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
      delete c;
      return fail(VB_EDEVICE, "hipStreamCreate failed: %s", hipGetErrorString(e));
    }
    c->own_stream = true;
  }
  register_ctx(c);
  *out = c;
  return VB_OK;
}

int vb_ctx_destroy(vb_ctx* c) {
  if (!c) return VB_OK;
  unregister_ctx(c);
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  c->release_side();
  if (c->own_stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return VB_OK;
}

int vb_ctx_synchronize(vb_ctx* c) {
  VB_TRY(check_ctx(c));
  return sync(c);
}

void* vb_ctx_stream(vb_ctx* c) { return c ? (void*)c->stream : nullptr; }

// ---------------------------------------------------------------------------
int vb_family_sample(vb_ctx* c, const vb_family* fam, const double* lam, int64_t n,
                     const vb_noise* noise, double* x_out) {
  VB_TRY(check_ctx(c));
  FamInfo fi;
  VB_TRY(check_family(fam, &fi));
  if (!lam || !x_out || !noise || n < 0) return fail(VB_EINVAL, "null argument");
  const size_t nd = (size_t)n * fi.D;
  if (fi.kind == VB_FAMILY_FR_T) {
    const bool host = noise->kind == VB_NOISE_HOST;
    if (host && !noise->eps) return fail(VB_EINVAL, "host noise requires eps");
    if (n == 0) return VB_OK;
    In dl, dn;
    Out dx;
    VB_TRY(dl.stage(c, 0, lam, fi.P));
    if (host) VB_TRY(dn.stage(c, 1, noise->eps, nd + n));
    VB_TRY(dx.stage(c, 2, x_out, nd));
    uint32_t k0, k1;
    key_of(noise->seed, &k0, &k1);
    vbk::FrWork* W;
    VB_TRY(fr_work(c, &W));
    VB_TRY(vbk::fr_sqrt(W, fi.D, dl.d, c->stream));
    const double *s, *z;
    VB_TRY(vbk::fr_draw(W, fi.D, n, fi.df, host ? dn.d : nullptr, k0, k1, noise->stream,
                        (uint32_t)noise->step, &s, &z, c->stream));
    VB_TRY(vbk::fr_transform(W, fi.D, n, dl.d, s, z, dx.d, c->stream));
    VB_TRY(dx.finish(c));
    return sync(c);
  }
  In dl, dn;
  Out dx;
  VB_TRY(dl.stage(c, 0, lam, 2 * (size_t)fi.D));
  if (noise->kind == VB_NOISE_HOST) {
    if (!noise->eps) return fail(VB_EINVAL, "host noise requires eps");
    if (ptr_class(noise->eps) < 0) return foreign_ptr_error(noise->eps);
    VB_TRY(dn.stage(c, 1, noise->eps, nd));
  }
  VB_TRY(dx.stage(c, 2, x_out, nd));
  uint32_t k0, k1;
  key_of(noise->seed, &k0, &k1);
  VB_HIP(vbk::launch_sample(fi.kind, fi.D, n, dl.d, fi.t_scale, fi.shape,
                            noise->kind == VB_NOISE_HOST ? dn.d : nullptr, k0, k1, noise->stream,
                            (uint32_t)noise->step, dx.d, c->stream));
  VB_TRY(dx.finish(c));
  return sync(c);
}

int vb_family_logdensity(vb_ctx* c, const vb_family* fam, const double* lam, const double* x,
                         int64_t n, double* out) {
  VB_TRY(check_ctx(c));
  FamInfo fi;
  VB_TRY(check_family(fam, &fi));
  if (!lam || !x || !out || n < 0) return fail(VB_EINVAL, "null argument");
  In dl, dxx;
  Out dout;
  if (fi.kind == VB_FAMILY_FR_T) {
    if (n == 0) return VB_OK;
    VB_TRY(dl.stage(c, 0, lam, fi.P));
    VB_TRY(dxx.stage(c, 1, x, (size_t)n * fi.D));
    VB_TRY(dout.stage(c, 2, out, (size_t)n));
    vbk::FrWork* W;
    VB_TRY(fr_work(c, &W));
    VB_TRY(vbk::fr_logdensity(W, fi.D, fi.df, fi.t_const, dl.d, dxx.d, n, dout.d, c->stream));
    VB_TRY(dout.finish(c));
    return sync(c);
  }
  VB_TRY(dl.stage(c, 0, lam, 2 * (size_t)fi.D));
  VB_TRY(dxx.stage(c, 1, x, (size_t)n * fi.D));
  VB_TRY(dout.stage(c, 2, out, (size_t)n));
  VB_HIP(vbk::launch_family_logdensity(fi.kind, fi.D, n, dl.d, fi.df, fi.t_const, dxx.d, dout.d,
                                       c->stream));
  VB_TRY(dout.finish(c));
  return sync(c);
}

int vb_family_moments(vb_ctx* c, const vb_family* fam, const double* lam, double* sigma_out,
                      double* eig_out) {
  VB_TRY(check_ctx(c));
  FamInfo fi;
  VB_TRY(check_family(fam, &fi));
  if (!lam) return fail(VB_EINVAL, "null argument");
  if (fi.kind != VB_FAMILY_FR_T)
    return fail(VB_EUNSUPPORTED, "vb_family_moments is for the full-rank family");
  const size_t dd = (size_t)fi.D * fi.D;
  In dl;
  Out ds, de;
  VB_TRY(dl.stage(c, 0, lam, fi.P));
  VB_TRY(ds.stage(c, 1, sigma_out, sigma_out ? dd : 0));
  VB_TRY(de.stage(c, 2, eig_out, eig_out ? (size_t)fi.D : 0));
  vbk::FrWork* W;
  VB_TRY(fr_work(c, &W));
  VB_TRY(vbk::fr_moments(W, fi.D, dl.d, ds.d, de.d, c->stream));
  VB_TRY(ds.finish(c));
  VB_TRY(de.finish(c));
  VB_TRY(sync(c));
  if (eig_out) {
    if (int rc = vbk::fr_info(W, c->stream)) return rc;
  }
  return VB_OK;
}

int vb_target_logdensity(vb_ctx* c, const vb_target* tgt, const double* x, int64_t n,
                         double* out, double* grad_out) {
  VB_TRY(check_ctx(c));
  if (!tgt) return fail(VB_EINVAL, "null target");
  VB_TRY(check_target(tgt, (int)tgt->dim));
  if (!x || !out || n < 0) return fail(VB_EINVAL, "null argument");
  const int D = (int)tgt->dim;
  In dxx;
  Out dout, dg;
  VB_TRY(dxx.stage(c, 0, x, (size_t)n * D));
  VB_TRY(dout.stage(c, 1, out, (size_t)n));
  VB_TRY(dg.stage(c, 2, grad_out, grad_out ? (size_t)n * D : 0));
  if (tgt->kind == VB_TARGET_CALLBACK) {
    if (n == 0) return VB_OK;
    vbk::FrWork* W;
    VB_TRY(fr_work(c, &W));
    VB_TRY(vbk::host_target_eval(W, host_of(tgt), D, n, dxx.d, dout.d, dg.d, c->stream));
  } else if (tgt->kind == VB_TARGET_CORR_GAUSS) {
    if (n == 0) return VB_OK;
    const double* tp;
    double tc;
    VB_TRY(target_params(c, 3, tgt, &tp, &tc));
    vbk::FrWork* W;
    VB_TRY(fr_work(c, &W));
    VB_TRY(vbk::fr_target(W, tgt->kind, D, n, tp, tc, dxx.d, dout.d, dg.d, c->stream));
  } else {
    VB_HIP(vbk::launch_target_logdensity(tgt->kind, D, n, dxx.d, dout.d, dg.d, c->stream));
  }
  VB_TRY(dout.finish(c));
  VB_TRY(dg.finish(c));
  return sync(c);
}

// ---------------------------------------------------------------------------
int vb_objective_value_grad(vb_ctx* c, const vb_family* fam, const vb_target* tgt,
                            const vb_objective* obj, const double* lam, const vb_noise* noise,
                            double* value, double* grad) {
  VB_TRY(check_ctx(c));
  FamInfo fi;
  VB_TRY(check_family(fam, &fi));
  VB_TRY(check_target(tgt, fi.D));
  if (!obj || !lam || !noise || !value || !grad) return fail(VB_EINVAL, "null argument");
  if (obj->n_samples < 1 || obj->n_samples > (1LL << 31))
    return fail(VB_EINVAL, "n_samples must be positive");
  if (obj->kind < VB_OBJ_KLVI || obj->kind > VB_OBJ_KLVI_PD)
    return fail(VB_EINVAL, "unknown objective %d", obj->kind);
  if (obj->kind == VB_OBJ_CHIVI && !(obj->alpha > 0))
    return fail(VB_EINVAL, "alpha must be positive");
  VB_TRY(require_fr(fi.kind, tgt->kind));
  if (fi.kind == VB_FAMILY_FR_T) return fr_objective(c, fi, tgt, obj, lam, noise, value, grad);
  const int D = fi.D, N = (int)obj->n_samples;
  const size_t P = 2 * (size_t)D;
  const bool host = noise->kind == VB_NOISE_HOST;
  if (host && !noise->eps) return fail(VB_EINVAL, "host noise requires eps");
  uint32_t k0, k1;
  key_of(noise->seed, &k0, &k1);
  In dl, dn;
  Out dg;
  VB_TRY(dl.stage(c, 0, lam, P));
  if (host) VB_TRY(dn.stage(c, 1, noise->eps, (size_t)N * D));
  VB_TRY(dg.stage(c, 2, grad, P));
  // device copy of lam that the kernels may read (they do not write in emit mode)
  VB_TRY(c->slot[3].reserve(P * sizeof(double)));
  VB_HIP(hipMemcpyAsync(c->slot[3].p, dl.d, P * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
  double* dval;
  VB_TRY(c->slot[4].reserve(sizeof(double) * 2));
  dval = c->slot[4].d();

  const bool pd = obj->kind == VB_OBJ_KLVI_PD;
  const bool sep = vbk::target_separable(tgt->kind) && obj->kind != VB_OBJ_CHIVI;
  const bool cb = tgt->kind == VB_TARGET_CALLBACK;
  if (sep && D > vbk::kBlockDMax) {
    vbk::SepArgs a{};
    a.D = D;
    a.N = N;
    a.W = 1;
    a.n_pairs = (D + 1) / 2;
    a.n_steps = 1;
    a.emit_grad = 1;
    a.pd = pd ? (fi.kind == VB_FAMILY_MF_T ? 2 : 1) : 0;
    a.step0 = 0;
    a.hist_start = 1LL << 62;
    a.rng_step0 = (long long)noise->step;
    a.n_waves = a.n_pairs;
    a.t_scale = fi.t_scale;
    a.shape = fi.shape;
    a.lam = c->slot[3].d();
    VB_TRY(c->slot[5].reserve(sizeof(double) * a.n_waves));
    a.vpart = c->slot[5].d();
    a.grad = dg.d;
    a.noise = host ? dn.d : nullptr;
    a.k0 = k0;
    a.k1 = k1;
    a.stream = noise->stream;
    VB_HIP(vbk::launch_sep(fi.kind, tgt->kind, host, a, c->stream));
    VB_HIP(vbk::launch_sep_values(a.vpart, 1, a.n_waves, sep_c0(fi, pd), dval, c->stream));
  } else if (D <= vbk::kBlockDMax && !cb) {
    vbk::BlockArgs a{};
    a.pf = block_pf_enabled();
    a.D = D;
    a.N = N;
    a.W = 1;
    a.P = (int)P;
    a.n_steps = 1;
    a.emit_grad = 1;
    a.chivi = obj->kind == VB_OBJ_CHIVI;
    a.pd = pd;
    a.step0 = 0;
    a.hist_start = 1LL << 62;
    a.n_iters = 1;
    a.n_hist = 0;
    a.rng_step0 = (long long)noise->step;
    a.alpha = obj->alpha;
    a.t_scale = fi.t_scale;
    a.shape = fi.shape;
    a.t_const = fi.t_const;
    a.df = fi.df;
    a.lam = c->slot[3].d();
    a.ring = nullptr;
    a.values = dval;
    a.grad = dg.d;
    a.noise = host ? dn.d : nullptr;
    a.k0 = k0;
    a.k1 = k1;
    a.stream = noise->stream;
    a.stream_stride = 1;
    if (!host && predraw_enabled(fi.kind)) {
      const bool need_lq = a.chivi || a.pd;
      VB_TRY(c->slot[6].reserve(sizeof(double) * (size_t)N * D));
      if (need_lq) VB_TRY(c->slot[7].reserve(sizeof(double) * (size_t)N));
      VB_HIP(vbk::launch_block_predraw(fi.kind, D, N, 1, 1, k0, k1, a.stream, 1, a.rng_step0,
                                       fi.t_scale, fi.shape, fi.df, fi.t_const, c->slot[6].d(),
                                       need_lq ? c->slot[7].d() : nullptr, c->stream));
      a.noise = c->slot[6].d();
      a.noise_lq = need_lq ? c->slot[7].d() : nullptr;
      VB_HIP(vbk::launch_block(fi.kind, tgt->kind, true, a, 1, c->stream));
    } else {
      VB_HIP(vbk::launch_block(fi.kind, tgt->kind, host, a, 1, c->stream));
    }
  } else {
    // CHIVI or a non-separable target at D > kBlockDMax: materialised path
    vbk::FrWork* W;
    VB_TRY(fr_work(c, &W));
    VB_TRY(vbk::mf_wide_value_grad(W, mf_spec(fi, tgt, obj), c->slot[3].d(), host ? dn.d : nullptr,
                                   k0, k1, noise->stream, (uint32_t)noise->step, dval, dg.d,
                                   c->stream));
  }
  VB_HIP(hipMemcpyAsync(value, dval, sizeof(double), hipMemcpyDeviceToHost, c->stream));
  VB_TRY(dg.finish(c));
  return sync(c);
}

// ---------------------------------------------------------------------------
}  // extern "C"

struct vb_run {
  vb_ctx* ctx = nullptr;
  FamInfo fi{};
  int tgt = 0, obj = 0;
  double alpha = 2.0;
  int N = 0, W = 10;
  long long nprob = 1, n_iters = 0, hist_start = 0, n_hist = 0, done = 0;
  double eps = 0.1;
  vbk::LrSched sched{};
  int opt = 0;  // vb_optimizer_kind
  bool sep = false;
  int n_waves = 0;
  int max_chunk = 256;
  DevBuf lam, ring, hist, values, vpart, noise, smooth;
  DevBuf noise_lq;  // pre-drawn log q partials (block kernel, predraw)
  DevBuf noise2, noise_lq2;  // the second chunk buffer of the overlapped pre-draw
  // full-rank family / wide mean-field: one value_grad + update per step
  bool fr = false, wide = false;
  vbk::FrSpec spec{};
  vbk::MfSpec mspec{};
  DevBuf tparams, grad;
  DevBuf backup;  // full rank: lambda and the adagrad window at the start of an advance
  long long fr_retries = 0;  // full rank: advances run again after a short warm root
  // launch timing (vb_run_set_timing): event pairs, reused; `ev_used` recorded
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> evs;
  std::vector<long long> ev_steps;
  size_t ev_used = 0;
  long long vals_n = 0;   // values in this run's progress snapshot (vb_run_values_async)
  ~vb_run() {
    for (auto& e : evs) {
      (void)hipEventDestroy(e.first);
      (void)hipEventDestroy(e.second);
    }
    if (ctx && ctx->vals_owner == this) ctx->vals_owner = nullptr;
  }
  // the pair for the next bracketed launch of k steps (nullptr: timing off)
  int next_event(long long k, std::pair<hipEvent_t, hipEvent_t>** out) {
    *out = nullptr;
    if (!timing) return VB_OK;
    if (ev_used == evs.size()) {
      std::pair<hipEvent_t, hipEvent_t> e{};
      VB_HIP(hipEventCreate(&e.first));
      VB_HIP(hipEventCreate(&e.second));
      evs.push_back(e);
      ev_steps.push_back(0);
    }
    ev_steps[ev_used] = k;
    *out = &evs[ev_used++];
    return VB_OK;
  }
};

extern "C" {

int vb_run_create(vb_ctx* c, const vb_family* fam, const vb_target* tgt, const vb_objective* obj,
                  const vb_adagrad_config* cfg, int64_t n_problems, const double* init,
                  vb_run** out) {
  VB_TRY(check_ctx(c));
  if (!out) return fail(VB_EINVAL, "null output pointer");
  *out = nullptr;
  FamInfo fi;
  VB_TRY(check_family(fam, &fi));
  VB_TRY(check_target(tgt, fi.D));
  VB_TRY(require_fr(fi.kind, tgt->kind));
  if (!obj || !cfg || !init) return fail(VB_EINVAL, "null argument");
  if (!(cfg->learning_rate > 0)) return fail(VB_EINVAL, "learning rate must be positive");
  if (!std::isnan(cfg->learning_rate_end) && cfg->learning_rate <= cfg->learning_rate_end)
    return fail(VB_EINVAL, "initial learning rate must be greater than final learning rate");
  if (cfg->optimizer < VB_OPT_ADAGRAD || cfg->optimizer > VB_OPT_ADAM_IA)
    return fail(VB_EINVAL, "unknown optimizer %d", cfg->optimizer);
  const bool ia = cfg->optimizer != VB_OPT_ADAGRAD;
  if (cfg->window < 1) return fail(VB_EINVAL, "window must be positive");
  if (cfg->n_iters < 0) return fail(VB_EINVAL, "n_iters must be non-negative");
  if (n_problems < 1) return fail(VB_EINVAL, "n_problems must be positive");
  if (obj->n_samples < 1 || obj->n_samples > (1LL << 31))
    return fail(VB_EINVAL, "n_samples must be positive");
  const int D = fi.D;
  const bool fr = fi.kind == VB_FAMILY_FR_T;
  if (obj->kind < VB_OBJ_KLVI || obj->kind > VB_OBJ_KLVI_PD)
    return fail(VB_EINVAL, "unknown objective %d", obj->kind);
  const bool sep = !fr && vbk::target_separable(tgt->kind) && obj->kind != VB_OBJ_CHIVI &&
                   (D > vbk::kBlockDMax);
  // D > kBlockDMax without the fused kernel (CHIVI, non-separable targets, IA
  // optimisers): the materialised mean-field path, one problem per run
  // (the fused kernels keep the adagrad window on chip: windows > 64 use the
  // materialised path, whose window lives in HBM)
  const bool big_window = !ia && cfg->window > 64;
  const bool wide = !fr && ((D > vbk::kBlockDMax && (!sep || ia)) ||
                            tgt->kind == VB_TARGET_CALLBACK || big_window);
  if (sep && n_problems != 1)
    return fail(VB_EUNSUPPORTED, "wide (D > %d) runs hold one problem per vb_run", vbk::kBlockDMax);

  vb_run* r = new (std::nothrow) vb_run();
  if (!r) return fail(VB_ENOMEM, "out of host memory");
  r->ctx = c;
  r->fi = fi;
  r->tgt = tgt->kind;
  r->obj = obj->kind;
  r->alpha = obj->alpha;
  r->N = (int)obj->n_samples;
  r->W = ia ? 2 : cfg->window;  // IA: the ring holds the two moment vectors
  r->opt = cfg->optimizer;
  r->nprob = n_problems;
  r->n_iters = cfg->n_iters;
  if (ia) {
    r->n_hist = std::min<long long>(cfg->n_iters, 100LL * cfg->window);
    r->hist_start = cfg->n_iters - r->n_hist;
  } else {
    r->hist_start = (3 * cfg->n_iters) / 4;
    r->n_hist = cfg->n_iters - r->hist_start;
  }
  r->eps = cfg->epsilon;
  r->sched = make_sched(cfg->n_iters, cfg->learning_rate, cfg->learning_rate_end);
  r->sep = sep && !wide;
  r->wide = wide;
  r->n_waves = (D + 1) / 2;
  const size_t P = fi.P;
  auto bail = [&](int rc) {
    delete r;
    return rc;
  };
  int rc;
  if (wide) {
    if ((rc = r->grad.reserve(sizeof(double) * P)) != VB_OK) return bail(rc);
    r->mspec = mf_spec(fi, tgt, obj);
  }
  if (fr) {
    r->fr = true;
    const double* tp;
    double tc;
    if ((rc = target_params(c, 1, tgt, &tp, &tc)) != VB_OK) return bail(rc);
    if (tp) {
      const size_t np = (size_t)tgt->n_params;
      if ((rc = r->tparams.reserve(sizeof(double) * np)) != VB_OK) return bail(rc);
      hipError_t e = hipMemcpyAsync(r->tparams.p, tp, sizeof(double) * np, hipMemcpyDeviceToDevice,
                                    c->stream);
      if (e != hipSuccess) return bail(fail(VB_EDEVICE, "hipMemcpy failed: %s", hipGetErrorString(e)));
    }
    r->spec = fr_spec(fi, tgt, obj, r->tparams.d(), tc);
    if ((rc = r->grad.reserve(sizeof(double) * P)) != VB_OK) return bail(rc);
  }
  if ((rc = r->lam.reserve(sizeof(double) * P * n_problems)) != VB_OK) return bail(rc);
  if ((rc = r->ring.reserve(sizeof(double) * P * r->W * n_problems)) != VB_OK) return bail(rc);
  if ((rc = r->hist.reserve(sizeof(double) * P * std::max<long long>(r->n_hist, 1) * n_problems)) != VB_OK)
    return bail(rc);
  if ((rc = r->values.reserve(sizeof(double) * std::max<long long>(r->n_iters, 1) * n_problems)) != VB_OK)
    return bail(rc);
  if ((rc = r->smooth.reserve(sizeof(double) * P * n_problems)) != VB_OK) return bail(rc);
  if (sep && (rc = r->vpart.reserve(sizeof(double) * r->n_waves * r->max_chunk)) != VB_OK)
    return bail(rc);
  In di;
  if ((rc = di.stage(c, 0, init, P * n_problems)) != VB_OK) return bail(rc);
  hipError_t e = hipMemcpyAsync(r->lam.p, di.d, sizeof(double) * P * n_problems,
                                hipMemcpyDeviceToDevice, c->stream);
  if (e == hipSuccess) e = hipMemsetAsync(r->ring.p, 0, sizeof(double) * P * r->W * n_problems, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) return bail(fail(VB_EDEVICE, "run init failed: %s", hipGetErrorString(e)));
  *out = r;
  return VB_OK;
}

// The per-step launches of full-rank / wide mean-field runs (one value_grad +
// update per step and problem), for steps [r->done, r->done + n_steps).
static int advance_fr_steps(vb_ctx* c, vb_run* r, int64_t n_steps, const vb_noise* noise,
                            bool host, const double* noise_base, size_t per_step, uint32_t k0,
                            uint32_t k1) {
  const size_t P = r->fi.P;
    vbk::FrWork* W;
    VB_TRY(fr_work(c, &W));
    const uint32_t stride = noise->stream_stride ? noise->stream_stride : 1;
    for (long long off = 0; off < n_steps; ++off) {
      const long long step = r->done + off;
      const double lr = r->sched.at(step);
      for (long long q = 0; q < r->nprob; ++q) {
        double* lam = r->lam.d() + q * P;
        const double* eps =
            host ? noise_base + ((size_t)q * n_steps + off) * per_step : nullptr;
        double* hrow = step >= r->hist_start
                           ? r->hist.d() + (q * r->n_hist + (step - r->hist_start)) * P
                           : nullptr;
        if (r->fr) {
          // one problem with Philox draws: the adagrad step rides in the step's last
          // kernel, which also prepares the next step of this advance (vb_fr.hip)
          const bool fuse = r->nprob == 1 && !host && r->opt == VB_OPT_ADAGRAD && fr_fuse_enabled();
          const vbk::MfUpdate up{r->ring.d() + q * P * r->W, r->W, step, lr, r->eps, hrow};
          const vbk::FrNext nx{off + 1 < n_steps, (uint32_t)(noise->step + off + 1)};
          VB_TRY(vbk::fr_value_grad(W, r->spec, lam, eps, k0, k1,
                                    noise->stream + (uint32_t)q * stride,
                                    (uint32_t)(noise->step + off),
                                    r->values.d() + q * r->n_iters + step, r->grad.d(), c->stream,
                                    r->nprob == 1 && step > 0, r, fuse ? &up : nullptr,
                                    fuse ? &nx : nullptr));
          if (fuse) continue;
        }
        if (!r->fr && r->opt == VB_OPT_ADAGRAD) {
          // gradient pass applies the adagrad step and writes the history row
          const vbk::MfUpdate up{r->ring.d() + q * P * r->W, r->W, step, lr, r->eps, hrow};
          VB_TRY(vbk::mf_wide_value_grad(W, r->mspec, lam, eps, k0, k1,
                                         noise->stream + (uint32_t)q * stride,
                                         (uint32_t)(noise->step + off),
                                         r->values.d() + q * r->n_iters + step, r->grad.d(),
                                         c->stream, &up));
          continue;
        }
        if (!r->fr)
          VB_TRY(vbk::mf_wide_value_grad(W, r->mspec, lam, eps, k0, k1,
                                         noise->stream + (uint32_t)q * stride,
                                         (uint32_t)(noise->step + off),
                                         r->values.d() + q * r->n_iters + step, r->grad.d(),
                                         c->stream));
        if (r->opt != VB_OPT_ADAGRAD) {
          VB_HIP(vbk::launch_ia_update(r->opt, (long long)P, lam, r->grad.d(),
                                       r->ring.d() + q * P * r->W, step, lr, r->eps, 0.0, hrow,
                                       c->stream));
        } else {
          VB_HIP(vbk::launch_adagrad_update((long long)P, lam, r->grad.d(),
                                            r->ring.d() + q * P * r->W, r->W, step, lr, r->eps,
                                            nullptr, c->stream, hrow));
        }
      }
    }
  return VB_OK;
}

int vb_run_advance(vb_run* r, int64_t n_steps, const vb_noise* noise) {
  HostTrace ht0;
  if (!r) return fail(VB_EINVAL, "null vb_run");
  vb_ctx* c = r->ctx;
  VB_TRY(check_ctx(c));
  if (!noise) return fail(VB_EINVAL, "null noise");
  if (n_steps < 0 || r->done + n_steps > r->n_iters)
    return fail(VB_EINVAL, "advance(%lld) past n_iters=%lld (done %lld)", (long long)n_steps,
                (long long)r->n_iters, (long long)r->done);
  if (n_steps == 0) return VB_OK;
  const bool host = noise->kind == VB_NOISE_HOST;
  const int D = r->fi.D, N = r->N;
  const size_t P = r->fi.P;
  const size_t per_step = (size_t)N * D + (r->fr ? (size_t)N : 0);
  if (host) {
    if (!noise->eps) return fail(VB_EINVAL, "host noise requires eps");
    if (ptr_class(noise->eps) < 0) return foreign_ptr_error(noise->eps);
    const size_t tot = per_step * n_steps * r->nprob;
    if (is_device_ptr(noise->eps)) {
      // used in place
    } else {
      VB_TRY(r->noise.reserve(tot * sizeof(double)));
      VB_HIP(hipMemcpyAsync(r->noise.p, noise->eps, tot * sizeof(double), hipMemcpyHostToDevice,
                            c->stream));
    }
  }
  const double* noise_base =
      host ? (is_device_ptr(noise->eps) ? noise->eps : r->noise.d()) : nullptr;
  uint32_t k0, k1;
  key_of(noise->seed, &k0, &k1);

  std::pair<hipEvent_t, hipEvent_t>* call_ev = nullptr;
  if (!r->sep) {
    VB_TRY(r->next_event(n_steps, &call_ev));
    if (call_ev) VB_HIP(hipEventRecord(call_ev->first, c->stream));
  }
  if (r->fr || r->wide) {
    // one full-rank problem: a snapshot of lambda and the adagrad window lets the
    // advance run again when a warm Newton-Schulz root launched too few
    // iterations (they launch exactly the learnt count, no spares; vb_fr.hip
    // fr_info)
    // (and the workspace's warm state: the rerun's first step starts from the
    // same previous root, power vectors and schedule as the failed pass did)
    const bool snap = r->fr && r->nprob == 1;
    const size_t snap_n = P + P * (size_t)r->W;
    vbk::FrWork* W = nullptr;
    if (r->fr) VB_TRY(fr_work(c, &W));
    if (snap) {
      VB_TRY(r->backup.reserve(snap_n * sizeof(double)));
      VB_HIP(hipMemcpyAsync(r->backup.d(), r->lam.d(), P * sizeof(double), hipMemcpyDeviceToDevice,
                            c->stream));
      VB_HIP(hipMemcpyAsync(r->backup.d() + P, r->ring.d(), P * r->W * sizeof(double),
                            hipMemcpyDeviceToDevice, c->stream));
      if (int rc = vbk::fr_warm_save(W, c->stream)) return rc;
    }
    // lambda and the adagrad window back to the snapshot (before a rerun, and
    // before returning an error: a failed advance leaves the run as it was)
    auto restore = [&]() -> int {
      VB_HIP(hipMemcpyAsync(r->lam.d(), r->backup.d(), P * sizeof(double),
                            hipMemcpyDeviceToDevice, c->stream));
      VB_HIP(hipMemcpyAsync(r->ring.d(), r->backup.d() + P, P * r->W * sizeof(double),
                            hipMemcpyDeviceToDevice, c->stream));
      return vbk::fr_warm_restore(W, c->stream);
    };
    // reruns of THIS advance: fr_info raises a count each time (Newton-Schulz by 3
    // up to kFrNSMax, PCG x2 up to kFrPcgMax) and reports an error past those, so
    // the loop ends by itself; the cap is a backstop.  r->fr_retries only counts
    // (vb_run_fr_retries).
    int reruns = 0;
    for (bool rerun = false;; rerun = true) {
      int rc = advance_fr_steps(c, r, n_steps, noise, host, noise_base, per_step, k0, k1);
      if (rc == VB_OK && r->fr) rc = sync(c);
      bool again = false;
      if (rc == VB_OK && r->fr) rc = vbk::fr_info(W, c->stream, snap ? &again : nullptr);
      if (rc == VB_OK && again && ++reruns > 32)
        rc = fail(VB_EDEVICE, "full-rank advance: too many reruns");
      if (rc != VB_OK) {
        if (snap) (void)restore();
        return rc;
      }
      if (!again) {
        if (rerun) vbk::fr_retry_done(W);
        break;
      }
      ++r->fr_retries;
      if (int rc2 = restore()) return rc2;
    }
  } else if (r->sep) {
    ht0.mark();
    ht0.print("advance entry -> sep branch");
    long long off = 0;
    while (off < n_steps) {
      const int cs = (int)std::min<long long>(r->max_chunk, n_steps - off);
      vbk::SepArgs a{};
      a.D = D;
      a.N = N;
      a.W = r->W;
      a.n_pairs = r->n_waves;
      a.n_steps = cs;
      a.emit_grad = 0;
      a.pd = r->obj == VB_OBJ_KLVI_PD ? (r->fi.kind == VB_FAMILY_MF_T ? 2 : 1) : 0;
      a.step0 = r->done + off;
      a.hist_start = r->hist_start;
      a.rng_step0 = (long long)noise->step + off;
      a.n_waves = r->n_waves;
      a.t_scale = r->fi.t_scale;
      a.shape = r->fi.shape;
      a.eps = r->eps;
      a.lr = r->sched;
      a.lam = r->lam.d();
      a.ring = r->ring.d();
      a.hist = r->hist.d();
      a.vpart = r->vpart.d();
      a.grad = nullptr;
      a.noise = host ? noise_base + (size_t)off * per_step : nullptr;
      a.k0 = k0;
      a.k1 = k1;
      a.stream = noise->stream;
      std::pair<hipEvent_t, hipEvent_t>* ev;
      HostTrace ht;
      VB_TRY(r->next_event(cs, &ev));
      ht.mark();
      // timed runs: the pair bracketed by event records (hipExtLaunchKernel's own
      // start / stop stamps instead measured ~0.2 us/step slower on the host path,
      // interleaved, profiles/r05/headline_ab_c.log)
      if (ev) VB_HIP(hipEventRecord(ev->first, c->stream));
      VB_HIP(vbk::launch_sep(r->fi.kind, r->tgt, host, a, c->stream));
      ht.mark();
      VB_HIP(vbk::launch_sep_values(a.vpart, cs, a.n_waves, sep_c0(r->fi, a.pd != 0),
                                    r->values.d() + a.step0, c->stream));
      if (ev) VB_HIP(hipEventRecord(ev->second, c->stream));
      ht.mark();
      ht.print("sep advance: next_event | record + launch_sep | launch_values + record");
      off += cs;
    }
  } else {
    vbk::BlockArgs a{};
    a.pf = block_pf_enabled();
    a.D = D;
    a.N = N;
    a.W = r->W;
    a.P = (int)P;
    a.n_steps = (int)n_steps;
    a.emit_grad = 0;
    a.chivi = r->obj == VB_OBJ_CHIVI;
    a.pd = r->obj == VB_OBJ_KLVI_PD;
    a.opt = r->opt;
    a.step0 = r->done;
    a.hist_start = r->hist_start;
    a.n_iters = r->n_iters;
    a.n_hist = r->n_hist;
    a.rng_step0 = (long long)noise->step;
    a.alpha = r->alpha;
    a.t_scale = r->fi.t_scale;
    a.shape = r->fi.shape;
    a.t_const = r->fi.t_const;
    a.df = r->fi.df;
    a.eps = r->eps;
    a.lr = r->sched;
    a.lam = r->lam.d();
    a.ring = r->ring.d();
    a.hist = r->hist.d();
    a.values = r->values.d();
    a.grad = nullptr;
    a.noise = noise_base;
    a.noise_lq = nullptr;
    a.k0 = k0;
    a.k1 = k1;
    a.stream = noise->stream;
    a.stream_stride = noise->stream_stride ? noise->stream_stride : 1;
    if (!host && predraw_enabled(r->fi.kind, true, N, D, a.chivi || a.pd)) {
      // Philox draws pre-drawn chunk by chunk by a throughput kernel over the
      // whole chip, then consumed through the device-noise path: the same
      // draws and log q partials, off the per-step critical path
      const bool need_lq = a.chivi || a.pd;
      const size_t per_step = (size_t)r->nprob * N * (D + (need_lq ? 1 : 0)) * sizeof(double);
      const long long cap = std::max<long long>(1, (long long)(kPredrawBytes / per_step));
      const int cmax = (int)std::min<long long>({n_steps, cap, (long long)kPredrawMaxSteps});
      const size_t nb = (size_t)r->nprob * cmax * N * D * sizeof(double);
      const size_t lb = (size_t)r->nprob * cmax * N * sizeof(double);
      VB_TRY(r->noise.reserve(nb));
      if (need_lq) VB_TRY(r->noise_lq.reserve(lb));
      // more than one chunk: chunk k + 1 is drawn on the odd CUs while the block
      // kernel runs chunk k on the even ones (two buffers, events between the
      // streams; the same draws and bits as the serial order)
      // (the streams are made on the first pre-drawn advance, whether or not it
      // overlaps: creating them costs milliseconds, paid outside later timed runs)
      const bool streams = predraw_overlap_enabled() && predraw_overlap_streams(c);
      // (several problems only: one problem's pre-draw is a few us per chunk, and
      // the cross-queue waits cost configs 1 / 2 ~3 %, profiles/r04/predraw_overlap_ab2.log)
      const bool overlap = n_steps > cmax && streams && r->nprob >= kPredrawOverlapMinProblems;
      if (overlap) {
        VB_TRY(r->noise2.reserve(nb));
        if (need_lq) VB_TRY(r->noise_lq2.reserve(lb));
      }
      hipStream_t pd_s = overlap ? c->pd_stream : c->stream;
      hipStream_t blk_s = overlap ? c->blk_stream : c->stream;
      hipEvent_t* ev = c->pd_ev;   // [0] start, [1..2] pre-draw of buffer b, [3..4] block of buffer b, [5] end
      if (overlap) {
        VB_HIP(hipEventRecord(ev[0], c->stream));
        VB_HIP(hipStreamWaitEvent(pd_s, ev[0], 0));
        VB_HIP(hipStreamWaitEvent(blk_s, ev[0], 0));
      }
      int k = 0;
      for (long long off = 0; off < n_steps; off += cmax, ++k) {
        const int cs = (int)std::min<long long>(cmax, n_steps - off);
        const int bsel = overlap ? (k & 1) : 0;
        double* nz = bsel ? r->noise2.d() : r->noise.d();
        double* nlq = need_lq ? (bsel ? r->noise_lq2.d() : r->noise_lq.d()) : nullptr;
        if (overlap && k >= 2) VB_HIP(hipStreamWaitEvent(pd_s, ev[3 + bsel], 0));  // buffer consumed
        VB_HIP(vbk::launch_block_predraw(r->fi.kind, D, N, cs, (int)r->nprob, k0, k1, a.stream,
                                         a.stream_stride, (long long)noise->step + off,
                                         r->fi.t_scale, r->fi.shape, r->fi.df, r->fi.t_const,
                                         nz, nlq, pd_s));
        if (overlap) {
          VB_HIP(hipEventRecord(ev[1 + bsel], pd_s));
          VB_HIP(hipStreamWaitEvent(blk_s, ev[1 + bsel], 0));
        }
        vbk::BlockArgs b = a;
        b.n_steps = cs;
        b.step0 = r->done + off;
        b.noise = nz;
        b.noise_lq = nlq;
        VB_HIP(vbk::launch_block(r->fi.kind, r->tgt, true, b, (int)r->nprob, blk_s));
        if (overlap) VB_HIP(hipEventRecord(ev[3 + bsel], blk_s));
      }
      if (overlap) {
        // the caller's stream resumes after both streams' work (the pre-draw stream
        // finished before the last block launch it fed)
        VB_HIP(hipEventRecord(ev[5], blk_s));
        VB_HIP(hipStreamWaitEvent(c->stream, ev[5], 0));
      }
    } else {
      VB_HIP(vbk::launch_block(r->fi.kind, r->tgt, host, a, (int)r->nprob, c->stream));
    }
  }
  if (call_ev) VB_HIP(hipEventRecord(call_ev->second, c->stream));
  r->done += n_steps;
  if (r->wide) return sync(c);
  if (r->fr) {
    VB_TRY(sync(c));
    vbk::FrWork* W;
    VB_TRY(fr_work(c, &W));
    if (int rc = vbk::fr_info(W, c->stream)) return rc;
    return VB_OK;
  }
  // host noise staging buffer is reused by the next call: finish before returning
  if (host) return sync(c);
  return VB_OK;
}

int vb_run_set_timing(vb_run* r, int enable) {
  if (!r) return fail(VB_EINVAL, "null vb_run");
  r->timing = enable != 0;
  return VB_OK;
}

int vb_run_launch_times(vb_run* r, int64_t max, int64_t* steps_out, float* ms_out,
                        int64_t* n_out) {
  if (!r || !n_out || (max > 0 && (!steps_out || !ms_out)))
    return fail(VB_EINVAL, "null argument");
  VB_TRY(check_ctx(r->ctx));
  const size_t n = std::min<size_t>(r->ev_used, (size_t)std::max<int64_t>(max, 0));
  for (size_t k = 0; k < n; ++k) {
    VB_HIP(hipEventSynchronize(r->evs[k].second));
    float ms = 0.f;
    VB_HIP(hipEventElapsedTime(&ms, r->evs[k].first, r->evs[k].second));
    steps_out[k] = r->ev_steps[k];
    ms_out[k] = ms;
  }
  *n_out = (int64_t)n;
  r->ev_used = 0;
  return VB_OK;
}

int vb_block_floor(vb_ctx* c, int32_t D, int32_t N, int32_t chivi, int32_t host_layout,
                   int64_t n_steps, int64_t n_problems, double* us_per_step) {
  VB_TRY(check_ctx(c));
  if (!us_per_step) return fail(VB_EINVAL, "null output pointer");
  if (D < 1 || D > vbk::kBlockDMax || N < 1 || n_steps < 1 || n_problems < 1 || n_problems > 65535)
    return fail(VB_EINVAL, "vb_block_floor: D in [1, %d], N >= 1, n_steps >= 1", vbk::kBlockDMax);
  DevBuf out;
  VB_TRY(out.reserve(sizeof(double) * n_problems));
  hipEvent_t e0, e1;
  VB_HIP(hipEventCreate(&e0));
  VB_HIP(hipEventCreate(&e1));
  VB_HIP(hipEventRecord(e0, c->stream));
  VB_HIP(vbk::launch_block_floor(D, N, host_layout != 0, chivi != 0, (int)n_steps,
                                 (int)n_problems, out.d(), c->stream, block_pf_enabled()));
  VB_HIP(hipEventRecord(e1, c->stream));
  VB_HIP(hipEventSynchronize(e1));
  float ms = 0.f;
  VB_HIP(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  *us_per_step = (double)ms * 1e3 / (double)n_steps;
  return VB_OK;
}

int vb_peak_probe(vb_ctx* c, int32_t kind, int64_t n, int32_t reps, double* out) {
  VB_TRY(check_ctx(c));
  if (!out) return fail(VB_EINVAL, "null output pointer");
  if (int rc = vbk::probe_rate(kind, (long long)n, reps, c->stream, out)) return rc;
  return VB_OK;
}

int vb_run_steps_done(vb_run* r, int64_t* out) {
  if (!r || !out) return fail(VB_EINVAL, "null argument");
  *out = r->done;
  return VB_OK;
}

int vb_run_fr_retries(vb_run* r, int64_t* out) {
  if (!r || !out) return fail(VB_EINVAL, "null argument");
  *out = r->fr_retries;
  return VB_OK;
}

int vb_run_result(vb_run* r, double* lam_out, double* hist_out, double* values_out,
                  double* smoothed_out) {
  if (!r) return fail(VB_EINVAL, "null vb_run");
  vb_ctx* c = r->ctx;
  VB_TRY(check_ctx(c));
  const size_t P = r->fi.P;
  auto copy_out = [&](double* dst, const void* src, size_t n) -> int {
    if (!dst || n == 0) return VB_OK;
    VB_HIP(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDefault, c->stream));
    return VB_OK;
  };
  VB_TRY(copy_out(lam_out, r->lam.p, P * r->nprob));
  VB_TRY(copy_out(hist_out, r->hist.p, P * r->n_hist * r->nprob));
  VB_TRY(copy_out(values_out, r->values.p, (size_t)r->n_iters * r->nprob));
  if (smoothed_out) {
    if (r->n_hist > 0) {
      VB_HIP(vbk::launch_row_mean(r->hist.d(), r->n_hist, (long long)P, r->nprob, r->smooth.d(),
                                  c->stream));
      VB_TRY(copy_out(smoothed_out, r->smooth.p, P * r->nprob));
    } else {
      // np.mean of an empty history is NaN (with a RuntimeWarning) in the reference
      std::vector<double> nanv(P * r->nprob, std::nan(""));
      VB_HIP(hipMemcpyAsync(smoothed_out, nanv.data(), nanv.size() * sizeof(double),
                            hipMemcpyDefault, c->stream));
      return sync(c);
    }
  }
  return sync(c);
}

int vb_run_values_async(vb_run* r, int64_t count) {
  if (!r) return fail(VB_EINVAL, "null vb_run");
  vb_ctx* c = r->ctx;
  VB_TRY(check_ctx(c));
  if (count < 0 || count > r->n_iters) return fail(VB_EINVAL, "count outside [0, n_iters]");
  const size_t need = std::max<size_t>(1, (size_t)count) * sizeof(double);
  if (need > c->vals_pin.cap) {
    // a snapshot still being copied into the old buffer lands before it goes
    if (c->vals_ev) VB_HIP(hipEventSynchronize(c->vals_ev));
    VB_TRY(c->vals_pin.reserve(std::max<size_t>(need, (size_t)r->n_iters * sizeof(double))));
  }
  if (!c->vals_ev) VB_HIP(hipEventCreateWithFlags(&c->vals_ev, hipEventDisableTiming));
  if (count > 0)
    VB_HIP(hipMemcpyAsync(c->vals_pin.p, r->values.p, (size_t)count * sizeof(double),
                          hipMemcpyDeviceToHost, c->stream));
  VB_HIP(hipEventRecord(c->vals_ev, c->stream));
  c->vals_owner = r;
  r->vals_n = count;
  return VB_OK;
}

int vb_run_values_wait(vb_run* r, double* out, int64_t* count_out) {
  if (!r || !out || !count_out) return fail(VB_EINVAL, "null argument");
  vb_ctx* c = r->ctx;
  VB_TRY(check_ctx(c));
  if (c->vals_owner != r)
    return fail(VB_EINVAL, "vb_run_values_wait: no snapshot of this run is pending (one per "
                           "context: a later vb_run_values_async of another run replaces it)");
  VB_HIP(hipEventSynchronize(c->vals_ev));
  if (r->vals_n > 0) std::memcpy(out, c->vals_pin.p, (size_t)r->vals_n * sizeof(double));
  *count_out = r->vals_n;
  return VB_OK;
}

int vb_run_destroy(vb_run* r) {
  if (!r) return VB_OK;
  if (r->ctx) {
    // the run's buffers go back to the device cache: nothing may still use them
    (void)hipSetDevice(r->ctx->device);
    (void)hipStreamSynchronize(r->ctx->stream);
    if (r->ctx->pd_stream) (void)hipStreamSynchronize(r->ctx->pd_stream);
    if (r->ctx->blk_stream) (void)hipStreamSynchronize(r->ctx->blk_stream);
  }
  delete r;
  return VB_OK;
}

int vb_adagrad_update(vb_ctx* c, int64_t P, double* lam, const double* grad, double* ring,
                      int32_t window, int64_t step, double lr, double epsilon) {
  VB_TRY(check_ctx(c));
  if (!lam || !grad || !ring || P < 1 || window < 1 || step < 0)
    return fail(VB_EINVAL, "invalid argument");
  if (!is_device_ptr(lam) || !is_device_ptr(ring))
    return fail(VB_EINVAL, "vb_adagrad_update keeps lam and ring on the device: pass device pointers");
  In dg;
  VB_TRY(dg.stage(c, 0, grad, (size_t)P));
  VB_HIP(vbk::launch_adagrad_update(P, lam, dg.d, ring, window, step, lr, epsilon, nullptr,
                                    c->stream));
  return sync(c);
}

int vb_adagrad_update_scaled(vb_ctx* c, int64_t P, double* lam, const double* grad, double* ring,
                             int32_t window, int64_t step, double lr, double epsilon,
                             const double* window_scale) {
  VB_TRY(check_ctx(c));
  if (!lam || !grad || !ring || !window_scale || P < 1 || window < 1 || step < 0)
    return fail(VB_EINVAL, "invalid argument");
  if (!is_device_ptr(lam) || !is_device_ptr(ring))
    return fail(VB_EINVAL, "vb_adagrad_update_scaled keeps lam and ring on the device: pass device pointers");
  const int64_t cnt = step + 1 < window ? step + 1 : window;
  In dg, dsc;
  VB_TRY(dg.stage(c, 0, grad, (size_t)P));
  VB_TRY(dsc.stage(c, 1, window_scale, (size_t)cnt));
  VB_HIP(vbk::launch_adagrad_update(P, lam, dg.d, ring, window, step, lr, epsilon, dsc.d,
                                    c->stream));
  return sync(c);
}

int vb_ia_update(vb_ctx* c, int32_t optimizer, int64_t P, double* lam, const double* grad,
                 double* state, int64_t step, double lr, double epsilon, double norm2,
                 double* old_out) {
  VB_TRY(check_ctx(c));
  if (!lam || !grad || !state || P < 1 || step < 0) return fail(VB_EINVAL, "invalid argument");
  if (optimizer != VB_OPT_RMSPROP_IA && optimizer != VB_OPT_ADAM_IA &&
      optimizer != VB_OPT_RMSPROP_IA_NORM)
    return fail(VB_EINVAL, "unknown optimizer %d", optimizer);
  if (!is_device_ptr(lam) || !is_device_ptr(state))
    return fail(VB_EINVAL, "vb_ia_update keeps lam and state on the device: pass device pointers");
  In dg;
  Out dold;
  VB_TRY(dg.stage(c, 0, grad, (size_t)P));
  VB_TRY(dold.stage(c, 1, old_out, old_out ? (size_t)P : 0));
  VB_HIP(vbk::launch_ia_update(optimizer, P, lam, dg.d, state, step, lr, epsilon, norm2, dold.d,
                               c->stream));
  VB_TRY(dold.finish(c));
  return sync(c);
}

// ---------------------------------------------------------------------------
int vb_log_weights_rows(vb_ctx* c, const vb_family* fam, const vb_target* tgt,
                        const double* lam, int64_t rows, int64_t m, const vb_noise* noise,
                        double* lw_out) {
  VB_TRY(check_ctx(c));
  FamInfo fi;
  VB_TRY(check_family(fam, &fi));
  VB_TRY(check_target(tgt, fi.D));
  if (!lam || !noise || !lw_out || m < 0 || rows < 0) return fail(VB_EINVAL, "null argument");
  if (rows > 65535) return fail(VB_EINVAL, "rows must be <= 65535");
  if (fi.kind == VB_FAMILY_FR_T) return fail(VB_EUNSUPPORTED, "rows of log weights: mean-field families only");
  if (noise->kind != VB_NOISE_PHILOX) return fail(VB_EINVAL, "rows of log weights need Philox noise");
  if ((!vbk::target_separable(tgt->kind) && fi.D > vbk::kBlockDMax) || tgt->kind == VB_TARGET_CALLBACK)
    return fail(VB_EUNSUPPORTED, "rows of log weights: D <= %d or a separable device target",
                vbk::kBlockDMax);
  if (m == 0 || rows == 0) return VB_OK;
  In dl;
  Out dlw;
  VB_TRY(dl.stage(c, 0, lam, 2 * (size_t)fi.D * rows));
  VB_TRY(dlw.stage(c, 2, lw_out, (size_t)m * rows));
  uint32_t k0, k1;
  key_of(noise->seed, &k0, &k1);
  VB_HIP(vbk::launch_log_weights(fi.kind, tgt->kind, fi.D, m, dl.d, fi.t_scale, fi.shape, fi.df,
                                 fi.t_const, nullptr, k0, k1, noise->stream,
                                 (uint32_t)noise->step, dlw.d, nullptr, c->stream, (int)rows,
                                 noise->stream_stride));
  VB_TRY(dlw.finish(c));
  return sync(c);
}

int vb_log_weights(vb_ctx* c, const vb_family* fam, const vb_target* tgt, const double* lam,
                   int64_t m, const vb_noise* noise, double* lw_out, double* samples_out) {
  VB_TRY(check_ctx(c));
  FamInfo fi;
  VB_TRY(check_family(fam, &fi));
  VB_TRY(check_target(tgt, fi.D));
  if (!lam || !noise || !lw_out || m < 0) return fail(VB_EINVAL, "null argument");
  VB_TRY(require_fr(fi.kind, tgt->kind));
  if (fi.kind == VB_FAMILY_FR_T) {
    const bool host = noise->kind == VB_NOISE_HOST;
    if (host && !noise->eps) return fail(VB_EINVAL, "host noise requires eps");
    if (m == 0) return VB_OK;
    In dl, dn;
    Out dlw, dxs;
    VB_TRY(dl.stage(c, 0, lam, fi.P));
    if (host) VB_TRY(dn.stage(c, 1, noise->eps, (size_t)m * fi.D + m));
    VB_TRY(dlw.stage(c, 2, lw_out, (size_t)m));
    VB_TRY(dxs.stage(c, 3, samples_out, samples_out ? (size_t)m * fi.D : 0));
    const double* tp;
    double tc;
    VB_TRY(target_params(c, 4, tgt, &tp, &tc));
    vbk::FrSpec f{};
    f.host = host_of(tgt);
    f.D = fi.D;
    f.tgt = tgt->kind;
    f.df = fi.df;
    f.t_const = fi.t_const;
    f.tparams = tp;
    f.tconst = tc;
    uint32_t k0, k1;
    key_of(noise->seed, &k0, &k1);
    vbk::FrWork* W;
    VB_TRY(fr_work(c, &W));
    VB_TRY(vbk::fr_log_weights(W, f, dl.d, m, host ? dn.d : nullptr, k0, k1, noise->stream,
                               (uint32_t)noise->step, dlw.d, dxs.d, c->stream));
    VB_TRY(dlw.finish(c));
    VB_TRY(dxs.finish(c));
    return sync(c);
  }
  if ((!vbk::target_separable(tgt->kind) && fi.D > vbk::kBlockDMax) ||
      tgt->kind == VB_TARGET_CALLBACK) {
    const bool host = noise->kind == VB_NOISE_HOST;
    if (host && !noise->eps) return fail(VB_EINVAL, "host noise requires eps");
    if (m == 0) return VB_OK;
    In dl, dn;
    Out dlw, dxs;
    VB_TRY(dl.stage(c, 0, lam, fi.P));
    if (host) VB_TRY(dn.stage(c, 1, noise->eps, (size_t)m * fi.D));
    VB_TRY(dlw.stage(c, 2, lw_out, (size_t)m));
    VB_TRY(dxs.stage(c, 3, samples_out, samples_out ? (size_t)m * fi.D : 0));
    uint32_t k0, k1;
    key_of(noise->seed, &k0, &k1);
    vbk::FrWork* W;
    VB_TRY(fr_work(c, &W));
    VB_TRY(vbk::mf_wide_log_weights(W, mf_spec(fi, tgt, nullptr), dl.d, m, host ? dn.d : nullptr,
                                    k0, k1, noise->stream, (uint32_t)noise->step, dlw.d, dxs.d,
                                    c->stream));
    VB_TRY(dlw.finish(c));
    VB_TRY(dxs.finish(c));
    return sync(c);
  }
  const bool host = noise->kind == VB_NOISE_HOST;
  if (host && !noise->eps) return fail(VB_EINVAL, "host noise requires eps");
  In dl, dn;
  Out dlw, dxs;
  VB_TRY(dl.stage(c, 0, lam, 2 * (size_t)fi.D));
  if (host) VB_TRY(dn.stage(c, 1, noise->eps, (size_t)m * fi.D));
  VB_TRY(dlw.stage(c, 2, lw_out, (size_t)m));
  VB_TRY(dxs.stage(c, 3, samples_out, samples_out ? (size_t)m * fi.D : 0));
  uint32_t k0, k1;
  key_of(noise->seed, &k0, &k1);
  VB_HIP(vbk::launch_log_weights(fi.kind, tgt->kind, fi.D, m, dl.d, fi.t_scale, fi.shape, fi.df,
                                 fi.t_const, host ? dn.d : nullptr, k0, k1, noise->stream,
                                 (uint32_t)noise->step, dlw.d, dxs.d, c->stream));
  VB_TRY(dlw.finish(c));
  VB_TRY(dxs.finish(c));
  return sync(c);
}

}  // extern "C"

// ---------------------------------------------------------------------------
extern "C" {

int vb_divergence_bound(vb_ctx* c, const double* lw, int64_t n, double alpha, int32_t has_elbo,
                        double elbo, double* out7) {
  VB_TRY(check_ctx(c));
  if (!lw || !out7) return fail(VB_EINVAL, "null argument");
  if (!(alpha > 1)) return fail(VB_EINVAL, "alpha must be greater than 1");  // bounds.py:166-167
  if (n < 1) return fail(VB_EINVAL, "log_weights must be non-empty");
  In dlw;
  VB_TRY(dlw.stage(c, 0, lw, (size_t)n));
  VB_TRY(c->slot[1].reserve(sizeof(double) * vbk::bounds_scratch_doubles(n, 1)));
  Out o;
  VB_TRY(o.stage(c, 2, out7, 7));
  VB_HIP(vbk::bounds_divergence(dlw.d, n, alpha, has_elbo, elbo, c->slot[1].d(), o.d, c->stream));
  VB_TRY(o.finish(c));
  return sync(c);
}

int vb_divergence_bound_rows(vb_ctx* c, const double* lw, int64_t rows, int64_t n, int64_t ld,
                             double alpha, int32_t has_elbo, double elbo, double* out7) {
  VB_TRY(check_ctx(c));
  if (!lw || !out7) return fail(VB_EINVAL, "null argument");
  if (!(alpha > 1)) return fail(VB_EINVAL, "alpha must be greater than 1");  // bounds.py:166-167
  if (n < 1) return fail(VB_EINVAL, "log_weights must be non-empty");
  if (rows < 1 || rows > 65535 || ld < n) return fail(VB_EINVAL, "invalid rows / ld");
  In dlw;
  VB_TRY(dlw.stage(c, 0, lw, (size_t)((rows - 1) * ld + n)));
  VB_TRY(c->slot[1].reserve(sizeof(double) * vbk::bounds_divergence_scratch_doubles(rows)));
  Out o;
  VB_TRY(o.stage(c, 2, out7, (size_t)rows * 7));
  VB_HIP(vbk::bounds_divergence_rows(dlw.d, rows, n, ld, alpha, has_elbo, elbo, c->slot[1].d(),
                                     o.d, c->stream));
  VB_TRY(o.finish(c));
  return sync(c);
}

int vb_centered_moments(vb_ctx* c, const double* x, int64_t n, int64_t d, double* c2,
                        double* c4) {
  VB_TRY(check_ctx(c));
  if (!x || !c2 || !c4 || n < 1 || d < 1) return fail(VB_EINVAL, "invalid argument");
  In dx;
  VB_TRY(dx.stage(c, 0, x, (size_t)n * d));
  VB_TRY(c->slot[1].reserve(sizeof(double) * vbk::bounds_scratch_doubles(n, d)));
  VB_TRY(c->slot[2].reserve(sizeof(double) * 2));
  VB_HIP(vbk::bounds_centered_moments(dx.d, n, d, c->slot[1].d(), c->slot[2].d(), c->stream));
  double h[2];
  VB_HIP(hipMemcpyAsync(h, c->slot[2].p, sizeof h, hipMemcpyDeviceToHost, c->stream));
  VB_TRY(sync(c));
  *c2 = h[0];
  *c4 = h[1];
  return VB_OK;
}

}  // extern "C"

// np.cov(x.T, aweights=w, ddof) / np.average with w raw weights or (logw) log
// weights normalised on the device as exp(lw - max lw); no O(n) host work
static int weighted_cov_impl(vb_ctx* c, const double* x, int64_t n, int64_t d, const double* w,
                             bool logw, int32_t ddof, double* mean_out, double* cov_out) {
  VB_TRY(check_ctx(c));
  if (!x || !cov_out || n < 1 || d < 1) return fail(VB_EINVAL, "invalid argument");
  if (d > (1LL << 30) || n > (1LL << 31)) return fail(VB_EINVAL, "sizes out of range");
  In dx, dw;
  VB_TRY(dx.stage(c, 0, x, (size_t)n * d));
  if (w) VB_TRY(dw.stage(c, 6, w, (size_t)n));
  VB_TRY(c->slot[1].reserve(sizeof(double) * vbk::bounds_wcov_scratch_doubles(n, d)));
  VB_TRY(c->slot[4].reserve(sizeof(double) * ((size_t)d + 8)));
  double* mdev = c->slot[4].d();
  double* sc = mdev + d;
  Out dm, dc;
  VB_TRY(dm.stage(c, 5, mean_out, mean_out ? (size_t)d : 0));
  VB_TRY(dc.stage(c, 2, cov_out, (size_t)d * d));
  VB_HIP(vbk::bounds_weighted_covariance(dx.d, n, d, w ? dw.d : nullptr, logw, ddof,
                                         c->slot[1].d(), sc, mdev, dc.d, c->stream));
  if (mean_out) VB_HIP(hipMemcpyAsync(dm.d, mdev, sizeof(double) * d, hipMemcpyDeviceToDevice, c->stream));
  double hsc[4] = {0.0, 0.0, 0.0, 1.0};
  if (w) VB_HIP(hipMemcpyAsync(hsc, sc, sizeof(hsc), hipMemcpyDeviceToHost, c->stream));
  VB_TRY(dm.finish(c));
  VB_TRY(dc.finish(c));
  VB_TRY(sync(c));
  if (!(hsc[3] > 0)) return fail(VB_EINVAL, "weights sum to zero");
  return VB_OK;
}

extern "C" {

int vb_weighted_covariance(vb_ctx* c, const double* x, int64_t n, int64_t d, const double* w,
                           int32_t ddof, double* mean_out, double* cov_out) {
  return weighted_cov_impl(c, x, n, d, w, false, ddof, mean_out, cov_out);
}

int vb_weighted_covariance_logw(vb_ctx* c, const double* x, int64_t n, int64_t d,
                                const double* log_w, int32_t ddof, double* mean_out,
                                double* cov_out) {
  if (!log_w) return fail(VB_EINVAL, "null log weights");
  return weighted_cov_impl(c, x, n, d, log_w, true, ddof, mean_out, cov_out);
}

int vb_covariance(vb_ctx* c, const double* x, int64_t n, int64_t d, double* mean_out,
                  double* cov_out) {
  VB_TRY(check_ctx(c));
  if (!x || !cov_out || n < 2 || d < 1) return fail(VB_EINVAL, "invalid argument");
  if (d > vbk::kCovDMax) return vb_weighted_covariance(c, x, n, d, nullptr, 1, mean_out, cov_out);
  In dx;
  VB_TRY(dx.stage(c, 0, x, (size_t)n * d));
  VB_TRY(c->slot[1].reserve(sizeof(double) * vbk::bounds_scratch_doubles(n, d)));
  Out dm, dc;
  VB_TRY(c->slot[4].reserve(sizeof(double) * d));
  double* mdev = c->slot[4].d();
  VB_TRY(dm.stage(c, 5, mean_out, mean_out ? (size_t)d : 0));
  VB_TRY(dc.stage(c, 2, cov_out, (size_t)d * d));
  VB_HIP(vbk::bounds_covariance(dx.d, n, d, c->slot[1].d(), mdev, dc.d, c->stream));
  if (mean_out) VB_HIP(hipMemcpyAsync(dm.d, mdev, sizeof(double) * d, hipMemcpyDeviceToDevice, c->stream));
  VB_TRY(dm.finish(c));
  VB_TRY(dc.finish(c));
  return sync(c);
}

}  // extern "C"

// ---------------------------------------------------------------------------
extern "C" {

// cutoff_ind = -ceil(min(0.2 n, 3 sqrt(n / Reff))) - 1   (psis.py:157)
static long long psis_tail_len(int64_t n, double reff) {
  return (long long)std::ceil(std::fmin(0.2 * (double)n, 3.0 * std::sqrt((double)n / reff)));
}

// m columns, element (i, col) at [col * cs + i * rs] of lw and lw_out; the
// columns run through the PSIS pipeline together (column-batched launches),
// in groups whose scratch stays within kPsisScratchBudget
static int psislw_impl(vb_ctx* c, const double* lw, int64_t n, int64_t m, long long rs,
                       long long cs, long long Mt, double* lw_out, double* k_out,
                       int64_t* tail_idx_out, int64_t tail_cap, int64_t* n_tail_out) {
  constexpr size_t kPsisScratchBudget = size_t(256) << 20;
  In dlw;
  VB_TRY(dlw.stage(c, 0, lw, (size_t)n * m));
  Out dout, dk;
  VB_TRY(dout.stage(c, 1, lw_out, (size_t)n * m));
  VB_TRY(dk.stage(c, 2, k_out, (size_t)m));
  const size_t sb = vbk::psis_col_stride(Mt < 1 ? 1 : Mt);
  const int64_t group = std::max<int64_t>(1, std::min<int64_t>(m, (int64_t)(kPsisScratchBudget / sb)));
  VB_TRY(c->slot[3].reserve(sb * (size_t)group));
  OutT<long long> dti, dnt;
  VB_TRY(dti.stage(c, 4, reinterpret_cast<long long*>(tail_idx_out),
                   tail_idx_out ? (size_t)tail_cap * m : 0));
  VB_TRY(c->slot[6].reserve(sizeof(unsigned) * (size_t)group));   // fast-select flags
  VB_TRY(c->psis_flags.reserve(sizeof(unsigned) * (size_t)group));  // their host copy
  VB_TRY(dnt.stage(c, 5, reinterpret_cast<long long*>(n_tail_out), n_tail_out ? (size_t)m : 0));
  for (int64_t c0 = 0; c0 < m; c0 += group) {
    const int g = (int)std::min<int64_t>(group, m - c0);
    VB_HIP(vbk::psis_columns(dlw.d + c0 * cs, dout.d ? dout.d + c0 * cs : nullptr, n, g, rs, cs,
                             Mt, c->slot[3].p,
                             dk.d + c0, dti.d ? dti.d + (size_t)c0 * tail_cap : nullptr,
                             (long long)tail_cap, dnt.d ? dnt.d + c0 : nullptr, c->stream,
                             static_cast<unsigned*>(c->slot[6].p),
                             static_cast<unsigned*>(c->psis_flags.p)));
  }
  VB_TRY(dout.finish(c));
  VB_TRY(dk.finish(c));
  VB_TRY(dti.finish(c));
  VB_TRY(dnt.finish(c));
  return sync(c);
}

int vb_psislw(vb_ctx* c, const double* lw, int64_t n, int64_t m, double reff, double* lw_out,
              double* k_out, int64_t* tail_idx_out, int64_t tail_cap, int64_t* n_tail_out) {
  VB_TRY(check_ctx(c));
  if (!lw || !k_out || m < 1) return fail(VB_EINVAL, "invalid argument");
  if (n <= 1) return fail(VB_EINVAL, "More than one log-weight needed.");  // psis.py:143-144
  const long long Mt = psis_tail_len(n, reff);
  if (Mt > vbk::psis_tail_max())
    return fail(VB_EUNSUPPORTED, "PSIS tail of %lld draws exceeds the device sort capacity %lld",
                Mt, vbk::psis_tail_max());
  if (tail_idx_out && tail_cap < Mt) return fail(VB_EINVAL, "tail_cap must be >= %lld", Mt);
  return psislw_impl(c, lw, n, m, /*rs=*/m, /*cs=*/1, Mt, lw_out, k_out, tail_idx_out, tail_cap,
                     n_tail_out);
}

int vb_psislw_colmajor(vb_ctx* c, const double* lw, int64_t n, int64_t m, double reff,
                       double* lw_out, double* k_out, int64_t* tail_idx_out, int64_t tail_cap,
                       int64_t* n_tail_out) {
  VB_TRY(check_ctx(c));
  if (!lw || !k_out || m < 1) return fail(VB_EINVAL, "invalid argument");
  if (n <= 1) return fail(VB_EINVAL, "More than one log-weight needed.");  // psis.py:143-144
  const long long Mt = psis_tail_len(n, reff);
  if (Mt > vbk::psis_tail_max())
    return fail(VB_EUNSUPPORTED, "PSIS tail of %lld draws exceeds the device sort capacity %lld",
                Mt, vbk::psis_tail_max());
  if (tail_idx_out && tail_cap < Mt) return fail(VB_EINVAL, "tail_cap must be >= %lld", Mt);
  return psislw_impl(c, lw, n, m, /*rs=*/1, /*cs=*/n, Mt, lw_out, k_out, tail_idx_out, tail_cap,
                     n_tail_out);
}

int vb_gpdfit(vb_ctx* c, const double* x, int64_t n, double* k, double* sigma, double* ks_out,
              double* w_out, int64_t* n_w_out) {
  VB_TRY(check_ctx(c));
  if (!x || !k || !sigma) return fail(VB_EINVAL, "null argument");
  if (n <= 1) return fail(VB_EINVAL, "Invalid input array.");  // psis.py:250-251
  if (n > vbk::psis_tail_max())
    return fail(VB_EUNSUPPORTED, "gpdfit of %lld values exceeds the device sort capacity %lld",
                (long long)n, vbk::psis_tail_max());
  const int m = 30 + (int)std::sqrt((double)n);
  In dx;
  VB_TRY(dx.stage(c, 0, x, (size_t)n));
  VB_TRY(c->slot[3].reserve(vbk::psis_scratch_bytes(n)));
  Out dks, dw;
  VB_TRY(dks.stage(c, 1, ks_out, ks_out ? (size_t)m : 0));
  VB_TRY(dw.stage(c, 2, w_out, w_out ? (size_t)m : 0));
  VB_TRY(c->slot[4].reserve(sizeof(double) * 4));
  VB_HIP(vbk::psis_gpdfit(dx.d, n, c->slot[3].p, c->slot[4].d(), dks.d, dw.d, c->stream));
  double h[4];
  VB_HIP(hipMemcpyAsync(h, c->slot[4].p, sizeof h, hipMemcpyDeviceToHost, c->stream));
  VB_TRY(dks.finish(c));
  VB_TRY(dw.finish(c));
  VB_TRY(sync(c));
  *k = h[0];
  *sigma = h[1];
  if (n_w_out) {
    long long nk;
    std::memcpy(&nk, &h[3], sizeof nk);
    *n_w_out = nk;
  }
  return VB_OK;
}

int vb_gpinv(vb_ctx* c, const double* p, int64_t n, double k, double sigma, double* out) {
  VB_TRY(check_ctx(c));
  if (!p || !out || n < 0) return fail(VB_EINVAL, "invalid argument");
  In dp;
  Out dout;
  VB_TRY(dp.stage(c, 0, p, (size_t)n));
  VB_TRY(dout.stage(c, 1, out, (size_t)n));
  VB_HIP(vbk::psis_gpinv(dp.d, n, k, sigma, dout.d, c->stream));
  VB_TRY(dout.finish(c));
  return sync(c);
}

// R-hat segments: job_len even, >= 2, inside [0, n_iters)
static int check_rhat_jobs(int64_t n_iters, int64_t n_jobs, const int64_t* job_start,
                           const int64_t* job_len) {
  for (int64_t j = 0; j < n_jobs; ++j) {
    if (job_len[j] < 2 || job_len[j] % 2 || (job_start && (job_start[j] < 0 ||
                                                           job_start[j] + job_len[j] > n_iters)))
      return fail(VB_EINVAL, "R-hat segment %lld: [%lld, +%lld) invalid for %lld iterations",
                  (long long)j, job_start ? (long long)job_start[j] : 0LL, (long long)job_len[j],
                  (long long)n_iters);
  }
  return VB_OK;
}

// the segments' starts and lengths in device memory (slot 1): [start | len]
static int rhat_jobs_dev(vb_ctx* c, int64_t n_jobs, const int64_t* job_start,
                         const int64_t* job_len, long long** dj) {
  VB_TRY(c->slot[1].reserve(sizeof(long long) * 2 * n_jobs));
  *dj = static_cast<long long*>(c->slot[1].p);
  if (job_start)
    VB_HIP(hipMemcpyAsync(*dj, job_start, sizeof(long long) * n_jobs, hipMemcpyHostToDevice,
                          c->stream));
  VB_HIP(hipMemcpyAsync(*dj + n_jobs, job_len, sizeof(long long) * n_jobs, hipMemcpyHostToDevice,
                        c->stream));
  return VB_OK;
}

int vb_rhat(vb_ctx* c, const double* chains, int64_t n_chains, int64_t n_iters, int64_t P,
            int64_t n_jobs, const int64_t* job_start, const int64_t* job_len, double* var_hat_out,
            double* rhat_out) {
  VB_TRY(check_ctx(c));
  if (!chains || !job_start || !job_len || !rhat_out) return fail(VB_EINVAL, "null argument");
  if (n_chains < 1 || n_iters < 0 || P < 1 || n_jobs < 0) return fail(VB_EINVAL, "invalid sizes");
  if (n_jobs == 0) return VB_OK;
  VB_TRY(check_rhat_jobs(n_iters, n_jobs, job_start, job_len));
  In dc;
  VB_TRY(dc.stage(c, 0, chains, (size_t)n_chains * n_iters * P));
  long long* dj;
  VB_TRY(rhat_jobs_dev(c, n_jobs, job_start, job_len, &dj));
  Out dv, dr;
  VB_TRY(dv.stage(c, 2, var_hat_out, var_hat_out ? (size_t)n_jobs * P : 0));
  VB_TRY(dr.stage(c, 3, rhat_out, (size_t)n_jobs * P));
  // the same two stages as the rank-sharded path (vb_rhat_stats on each rank's
  // chains, one gather, vb_rhat_combine), so both give the same bits
  const size_t ns = (size_t)n_jobs * 2 * n_chains * P;
  VB_TRY(c->slot[4].reserve(sizeof(double) * 2 * ns));
  double* st = c->slot[4].d();
  VB_HIP(vbk::launch_rhat_stats(dc.d, n_chains, n_iters, P, n_jobs, dj, dj + n_jobs, st, st + ns,
                                c->stream));
  VB_HIP(vbk::launch_rhat_combine(st, st + ns, 2 * n_chains, P, n_jobs, dj + n_jobs, dv.d, dr.d,
                                  c->stream));
  VB_TRY(dv.finish(c));
  VB_TRY(dr.finish(c));
  return sync(c);
}

int vb_rhat_stats(vb_ctx* c, const double* chains, int64_t n_chains, int64_t n_iters, int64_t P,
                  int64_t n_jobs, const int64_t* job_start, const int64_t* job_len,
                  double* mean_out, double* ss_out) {
  VB_TRY(check_ctx(c));
  if (!chains || !job_start || !job_len || !mean_out || !ss_out)
    return fail(VB_EINVAL, "null argument");
  if (n_chains < 1 || n_iters < 0 || P < 1 || n_jobs < 0) return fail(VB_EINVAL, "invalid sizes");
  if (n_jobs == 0) return VB_OK;
  VB_TRY(check_rhat_jobs(n_iters, n_jobs, job_start, job_len));
  In dc;
  VB_TRY(dc.stage(c, 0, chains, (size_t)n_chains * n_iters * P));
  long long* dj;
  VB_TRY(rhat_jobs_dev(c, n_jobs, job_start, job_len, &dj));
  const size_t ns = (size_t)n_jobs * 2 * n_chains * P;
  Out dm, dss;
  VB_TRY(dm.stage(c, 2, mean_out, ns));
  VB_TRY(dss.stage(c, 3, ss_out, ns));
  VB_HIP(vbk::launch_rhat_stats(dc.d, n_chains, n_iters, P, n_jobs, dj, dj + n_jobs, dm.d, dss.d,
                                c->stream));
  VB_TRY(dm.finish(c));
  VB_TRY(dss.finish(c));
  return sync(c);
}

int vb_rhat_combine(vb_ctx* c, const double* mean, const double* ss, int64_t n_halves, int64_t P,
                    int64_t n_jobs, const int64_t* job_len, double* var_hat_out, double* rhat_out) {
  VB_TRY(check_ctx(c));
  if (!mean || !ss || !job_len || !rhat_out) return fail(VB_EINVAL, "null argument");
  if (n_halves < 2 || n_halves % 2 || P < 1 || n_jobs < 0) return fail(VB_EINVAL, "invalid sizes");
  if (n_jobs == 0) return VB_OK;
  VB_TRY(check_rhat_jobs(0, n_jobs, nullptr, job_len));
  const size_t ns = (size_t)n_jobs * n_halves * P;
  In dm, dss;
  VB_TRY(dm.stage(c, 0, mean, ns));
  VB_TRY(dss.stage(c, 4, ss, ns));
  long long* dj;
  VB_TRY(rhat_jobs_dev(c, n_jobs, nullptr, job_len, &dj));
  Out dv, dr;
  VB_TRY(dv.stage(c, 2, var_hat_out, var_hat_out ? (size_t)n_jobs * P : 0));
  VB_TRY(dr.stage(c, 3, rhat_out, (size_t)n_jobs * P));
  VB_HIP(vbk::launch_rhat_combine(dm.d, dss.d, n_halves, P, n_jobs, dj + n_jobs, dv.d, dr.d,
                                  c->stream));
  VB_TRY(dv.finish(c));
  VB_TRY(dr.finish(c));
  return sync(c);
}

int vb_iterate_average(vb_ctx* c, const double* x, int64_t n, int64_t ld, int64_t cols,
                       int64_t start, double* out) {
  VB_TRY(check_ctx(c));
  if (!x || !out) return fail(VB_EINVAL, "null argument");
  if (n - start <= 0)  // functions.py:70-71
    return fail(VB_EINVAL, "Start of stationary distribution must be lower than number of iterates");
  if (start < 0 || cols < 1 || ld < cols) return fail(VB_EINVAL, "invalid sizes");
  In dx;
  VB_TRY(dx.stage(c, 0, x, (size_t)(n - 1) * ld + cols));
  Out dout;
  VB_TRY(dout.stage(c, 1, out, (size_t)(n - start) * cols));
  VB_HIP(vbk::launch_iterate_average(dx.d, n, ld, cols, start, dout.d, c->stream));
  VB_TRY(dout.finish(c));
  return sync(c);
}

int vb_sumlogs_rows(vb_ctx* c, const double* x, int64_t rows, int64_t n, double* out) {
  VB_TRY(check_ctx(c));
  if (!x || !out || n < 1 || rows < 1) return fail(VB_EINVAL, "invalid argument");
  In dx;
  VB_TRY(dx.stage(c, 0, x, (size_t)rows * n));
  VB_TRY(c->slot[3].reserve(vbk::psis_sumlogs_rows_scratch_bytes(rows, n)));
  Out dout;
  VB_TRY(dout.stage(c, 1, out, (size_t)rows));
  VB_HIP(vbk::psis_sumlogs_rows(dx.d, rows, n, c->slot[3].p, dout.d, c->stream));
  VB_TRY(dout.finish(c));
  return sync(c);
}

int vb_sumlogs(vb_ctx* c, const double* x, int64_t n, double* out) {
  VB_TRY(check_ctx(c));
  if (!x || !out || n < 1) return fail(VB_EINVAL, "invalid argument");
  In dx;
  VB_TRY(dx.stage(c, 0, x, (size_t)n));
  VB_TRY(c->slot[3].reserve(vbk::psis_scratch_bytes(0)));
  VB_TRY(c->slot[4].reserve(sizeof(double)));
  VB_HIP(vbk::psis_sumlogs(dx.d, n, c->slot[3].p, c->slot[4].d(), c->stream));
  VB_HIP(hipMemcpyAsync(out, c->slot[4].p, sizeof(double), hipMemcpyDeviceToHost, c->stream));
  return sync(c);
}

}  // extern "C"
