// fc_capi.hip — extern "C" entry points of libfedcodec.so (declared in include/fedcodec.h).
// Argument checking, sampling plans and launch sequences; no allocation, no host syncs.
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

// Part of the unity build (fedcodec.hip): the kernels and their argument structs from
// fc_topk.hip / fc_decode.hip are visible here.
#include <hip/hip_ext.h>

#include "fc_state.h"

using namespace fc;

static thread_local char g_err[512];

static int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}

#define FC_CHECK(cond, ...) \
  do { if (!(cond)) return fail(FC_ERR_ARG, __VA_ARGS__); } while (0)
#define FC_LAUNCHED(name)                                                          \
  do {                                                                             \
    hipError_t e_ = hipGetLastError();                                             \
    if (e_ != hipSuccess) return fail(FC_ERR_HIP, "%s: %s", name, hipGetErrorString(e_)); \
  } while (0)

static uint32_t index_bits(uint64_t n) {
  uint32_t b = 1;
  while (b < 32 && (1ull << b) < n) ++b;
  return b;
}

static uint32_t num_chunks(uint64_t n) { return (uint32_t)((n + kChunk - 1) / kChunk); }

static WsPtrs ws_ptrs(void* ws, uint64_t n) {
  const WsLayout L = WsLayout::of(n);
  char* b = static_cast<char*>(ws);
  WsPtrs W;
  W.st = reinterpret_cast<TopkState*>(b);
  W.hist1 = reinterpret_cast<uint32_t*>(b + L.off_hist1);
  W.tick = reinterpret_cast<uint32_t*>(b + L.off_tick);
  W.ehist = reinterpret_cast<uint32_t*>(b + L.off_ehist);
  W.chist = reinterpret_cast<uint32_t*>(b + L.off_chist);
  W.small = reinterpret_cast<uint64_t*>(b + L.off_small);
  W.smallv = reinterpret_cast<uint32_t*>(b + L.off_smallv);
  W.pub = reinterpret_cast<uint32_t*>(b + L.off_pub);
  W.ccnt = reinterpret_cast<uint32_t*>(b + L.off_status);
  W.cand = reinterpret_cast<uint64_t*>(b + L.off_cand);
  W.cand_cap = L.cand_cap;
  return W;
}

// Stratified sample + bracket ranks.  Full sample for n <= 1 M (exact bracket); otherwise
// 64..1024 segments of 1024 (n/64 .. 1 M keys) and a +-6 sigma binomial margin.
// Decode grid: per_cu workgroups per CU (capped at one per chunk), each walking
// ceil(chunks / grid) chunks.  FC_DECODE_GRID overrides it in FC_DEBUG_BUILD libraries only
// (tuning); the shipped library's geometry never depends on the host environment.
static uint32_t decode_grid(uint64_t n, uint32_t per_cu = kDecBlocksPerCU) {
#ifdef FC_DEBUG_BUILD
  static const uint32_t forced = [] {
    const char* e = getenv("FC_DECODE_GRID");
    return e ? (uint32_t)atoi(e) : 0u;
  }();
#else
  constexpr uint32_t forced = 0;
#endif
  uint32_t g = forced ? forced : 256u * per_cu;
  const uint32_t nch = num_chunks(n);
  return g < nch ? g : nch;
}

constexpr int FC_MAX_SAMPLE_SEGS = 1024;
constexpr int FC_SAMPLE_DIV = 64;                          // sample 1/64 of the gradient (below the cap)
// fc_topk_encode_dense (the drop-in compress('top') path) samples more: its sample latency
// hides under the fused launch's first round of chunk loads, and a narrower bracket means
// fewer candidates on its critical path (16 M: 256 -> 512 segments took 68.8 -> 60.8 us; the
// 128-client bench step got slower with a bigger sample: profiles/r02_ab_sample_plan.jsonl).
// Its dense result does not depend on the bracket; packet encodes keep the batched plan, so a
// single encode_top and a batched one write the same packet bytes (slack included).
constexpr int FC_SAMPLE_DIV_SINGLE = 32;
constexpr int FC_MAX_SAMPLE_SEGS_SINGLE = 2048;
constexpr int FC_SAMPLE_ROUNDS = 4;                        // sample groups per batched k_sample1 workgroup
// Candidate-histogram bins a batched encode's bracket is cut into: ~kCandPerBin expected
// candidates per bin, 256..4096 bins.  Every batched resolve workgroup flushes that many
// coalesced bins and the survivors of one bin are sorted on the chain, so fewer, fuller bins
// suit a small gradient (configs[2], 16 M: ~120 K candidates -> 1024 bins, resolve 97 -> 86 us
// per 128-client step) and 4096 a large one (128 M: ~465 K; 1024 bins made the batched
// resolve slower, 151 -> 158 us per 64 clients, profiles/r05_ab_cand_bins.jsonl).  A lone
// encode keeps 4096: its compaction bins every candidate with a device atomic, and fewer bins
// queue more of them on one address (128 M packet encode 167 -> 277 us with 1024).
constexpr int FC_CAND_PER_BIN = 128;
static uint32_t cand_bins_log2(uint64_t n, const SamplePlan& P) {
  if (P.full || P.lo_all || P.hi_none) return 12;
  const double S = (double)P.nseg * 1024.0;
  const double expect = (double)(P.r_lo - P.r_hi) * (double)n / S;   // candidates in the bracket
  uint32_t lg = 8;
  while (lg < 12 && (double)(1u << lg) * FC_CAND_PER_BIN < expect) ++lg;
  return lg;
}
static SamplePlan make_plan(uint64_t n, uint64_t k, bool single = false) {
  SamplePlan P;
  memset(&P, 0, sizeof P);
  P.n = n;
  if (n <= kFullSampleMax) {
    P.full = 1;
    P.nseg = (uint32_t)((n + 1023) / 1024);
    P.r_hi = P.r_lo = (int64_t)k;
  } else {
    // 1/64 of the gradient, 64..1024 segments: at 16 M a 64-client batch spends 1391 us in
    // sample + compact + resolve with 256 segments against 1481 us with 512 (1/32)
    uint64_t seg = n / (single ? FC_SAMPLE_DIV_SINGLE : FC_SAMPLE_DIV) / 1024;
    if (seg < 64) seg = 64;
    const uint64_t cap = single ? FC_MAX_SAMPLE_SEGS_SINGLE : FC_MAX_SAMPLE_SEGS;
    if (seg > cap) seg = cap;
    P.nseg = (uint32_t)seg;
    const double S = (double)seg * 1024.0;
    const double q = (double)k / (double)n;
    const double rho = q * S;
    const double m = 6.0 * sqrt(S * q * (1.0 - q)) + 16.0;
    P.r_hi = (int64_t)floor(rho - m);
    P.r_lo = (int64_t)ceil(rho + m);
    if (P.r_lo > (int64_t)S) P.lo_all = 1;
  }
  if (P.r_hi < 1) P.hi_none = 1;
  P.cbins_log2 = 12;                 // lone encodes (fused in-kernel binning); batched: below
  // pilot (k_sample1): kPilotSegs segments spread over the sample, read by every workgroup.
  // Its ranks bracket the sample ranks scaled to the pilot, widened by 7 pilot sigmas + 8.
  P.segs = n <= (32ull << 20) ? 2u : (uint32_t)kSampleSegs;
  P.pstride = (P.nseg + P.segs - 1) / P.segs;                    // the sample grid
  P.np = 0;
  while (P.np < P.segs && P.np * P.pstride < P.nseg) ++P.np;
  double Sp = 0.0;
  for (uint32_t j = 0; j < P.np; ++j) {
    const uint64_t st = seg_start(P, pilot_seg(P, j));
    const uint64_t lim = P.full ? std::min<uint64_t>(st + 1024, n) : st + 1024;
    Sp += (double)(lim - st);
  }
  const double S = P.full ? (double)n : (double)P.nseg * 1024.0;
  const double q = (double)k / (double)n;
  const double sig = sqrt(Sp * q * (1.0 - q));
  const int64_t isp = (int64_t)Sp;
  P.pr_hi = std::max<int64_t>(1, (int64_t)floor((double)P.r_hi * Sp / S - 7.0 * sig - 8.0));
  P.pr_lo = std::min<int64_t>(isp, (int64_t)ceil((double)P.r_lo * Sp / S + 7.0 * sig + 8.0));
  if (P.pr_hi > isp) P.pr_hi = isp;
  if (P.pr_lo < P.pr_hi) P.pr_lo = P.pr_hi;
  return P;
}

static int check_common(const float* g, uint64_t n, void* ws, size_t ws_bytes) {
  FC_CHECK(g != nullptr, "g is NULL");
  FC_CHECK(n >= 1 && n <= 0xffffffffull, "n=%llu outside [1, 2^32-1]", (unsigned long long)n);
  FC_CHECK(((uintptr_t)g & 15) == 0, "g must be 16-byte aligned");
  FC_CHECK(ws != nullptr, "workspace is NULL");
  if (ws_bytes < WsLayout::of(n).bytes)
    return fail(FC_ERR_WORKSPACE, "workspace %zu B < %llu B needed", ws_bytes,
                (unsigned long long)WsLayout::of(n).bytes);
  return FC_OK;
}

// ---- opt-in kernel timing (fc_timing_begin / fc_timing_end) ------------------------------
namespace {
struct EvPair { hipEvent_t a, b; uint32_t cat; };
std::vector<EvPair> g_ev;
size_t g_ev_used = 0;
uint32_t g_time_mask = 0;

// Brackets one launch with a hipEvent pair on its own stream when its class is selected.
struct TimedLaunch {
  long slot = -1;
  hipStream_t s;
  TimedLaunch(uint32_t cat, hipStream_t s_) : s(s_) {
    if (!(g_time_mask & cat)) return;
    if (g_ev_used == g_ev.size()) {
      EvPair e{nullptr, nullptr, 0};
      if (hipEventCreate(&e.a) != hipSuccess || hipEventCreate(&e.b) != hipSuccess) return;
      g_ev.push_back(e);
    }
    slot = (long)g_ev_used++;
    g_ev[slot].cat = cat;
    (void)hipEventRecord(g_ev[slot].a, s);
  }
  ~TimedLaunch() { if (slot >= 0) (void)hipEventRecord(g_ev[slot].b, s); }
};
}  // namespace

// k_sample1 for one client (jobs == nullptr) or a batch (grid.y = clients).
static int launch_sample(int key_mode, dim3 grid, const float* g, const SamplePlan& P,
                         uint64_t seed, uint64_t offset, const WsPtrs& W, uint32_t ib,
                         fc_packet_hdr* hdr, const HdrInit& hi, const fc_encode_job* jobs,
                         uint64_t stride, hipStream_t s) {
  TimedLaunch t(FC_TIME_SAMPLE, s);
  if (key_mode == FC_KEY_PHILOX) {
    hipLaunchKernelGGL(k_sample1<kKeyPhilox>, grid, dim3(kBlock), 0, s, g, P, seed, offset, W, ib, hdr, hi, jobs, stride);
  } else if (jobs) {                 // batched: one pilot per client, then the sample
    hipLaunchKernelGGL(k_pilot<kKeyMag>, dim3(grid.y), dim3(kBlock), 0, s, P, W, jobs, stride);
    FC_LAUNCHED("k_pilot");
    hipLaunchKernelGGL((k_sample1<kKeyMag, true>), grid, dim3(kBlock), 0, s, g, P, seed, offset, W, ib, hdr, hi, jobs, stride);
  } else {
    hipLaunchKernelGGL(k_sample1<kKeyMag>, grid, dim3(kBlock), 0, s, g, P, seed, offset, W, ib, hdr, hi, jobs, stride);
  }
  FC_LAUNCHED("k_sample1");
  return FC_OK;
}

static int launch_engine(int key_mode, const EngineArgs& base, int passes, hipStream_t s) {
#ifdef FC_DEBUG_BUILD
  if (const char* dbg = getenv("FC_DEBUG_ENGINE_PASSES")) passes = atoi(dbg);  // debug builds only
#endif
  for (int p = 0; p < passes; ++p) {
    TimedLaunch t(FC_TIME_ENGINE, s);
    EngineArgs a = base;
    a.first = p == 0;
    if (key_mode == FC_KEY_PHILOX) hipLaunchKernelGGL(k_engine<kKeyPhilox>, dim3(kEngineGrid), dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL(k_engine<kKeyMag>, dim3(kEngineGrid), dim3(kBlock), 0, s, a);
    FC_LAUNCHED("k_engine");
  }
  return FC_OK;
}

// top-k compaction: k_compact_mag1, one workgroup per (chunk, client).  (Measured slower
// and dropped: a persistent LDS-DMA ring, 1.5x; one wave per chunk, 1.1x — DESIGN.md §Lessons.)
// (mag_item_of: a 3-D grid of interleave groups, or a linear one past the grid's y limit)
static dim3 compact_mag_grid(CompactArgs& a, uint32_t m) {
  a.m = m;
  const uint32_t il = m < (uint32_t)FC_MAG1_IL ? m : (uint32_t)FC_MAG1_IL;
  a.grid3 = a.nchunks <= 65535u ? 1u : 0u;
  return a.grid3 ? dim3(il, a.nchunks, (m + il - 1) / il) : dim3(a.nchunks, m);
}
static void launch_compact_mag(const CompactArgs& a, uint32_t m, hipStream_t s) {
  CompactArgs b = a;
  const dim3 grid = compact_mag_grid(b, m);
  hipLaunchKernelGGL(k_compact_mag1, grid, dim3(kCBlock), 0, s, b);
}

// the PredArgs of k_compact_pred from a compaction's CompactArgs
static PredArgs pred_args(const CompactArgs& a) {
  PredArgs p;
  memset(&p, 0, sizeof p);
  p.g = a.g; p.n = a.n; p.seed = a.seed; p.offset = a.offset; p.bern_thr = a.bern_thr;
  p.mask = a.mask; p.idx = a.idx; p.val = a.val; p.bitmap = a.bitmap; p.cnt = a.cnt;
  p.qoff = a.qoff; p.S = a.W.st; p.ccnt = a.W.ccnt; p.cand = a.W.cand; p.jobs = a.jobs;
  p.ws_stride = a.ws_stride; p.ib = a.ib; p.nonfinite_keep = a.nonfinite_keep;
  return p;
}

// bin: a lone rand-k compaction also fills the candidate histogram (k_resolve<false> follows alone)
static int launch_compact_key(int key_mode, const CompactArgs& a, hipStream_t s, uint32_t m = 1,
                              bool bin = false) {
  TimedLaunch t(FC_TIME_COMPACT, s);
  if (key_mode == FC_KEY_PHILOX) {
    PredArgs p = pred_args(a);
    if (bin) p.chist = a.W.chist;
    hipLaunchKernelGGL((k_compact_pred<kSrcPhiloxKey, FC_FMT_IDXVAL>), dim3(a.nchunks, m), dim3(kCBlock), 0, s, p);
  } else {
    launch_compact_mag(a, m, s);
  }
  FC_LAUNCHED("k_compact");
  return FC_OK;
}

// Native rand-k: the keys (Philox word >> 1) are uniform on [0, 2^31), so #(key > t) is
// Binomial(n, (2^31 - 1 - t) / 2^31) and the bracket around the k-th key needs no sample:
// t_hi puts k - 8 sigma - 16 keys above it on average, t_lo k + 8 sigma + 16 at or above it
// (a miss is ~1e-15 likely and only costs the exact re-encode).  ~16 sigma candidates.
static void philox_bracket(uint64_t n, uint64_t k, uint32_t* t_lo, uint32_t* t_hi, uint32_t* sbin) {
  const double N = (double)n, K = (double)k, R = 2147483648.0;
  const double M = 8.0 * sqrt(K * (1.0 - K / N)) + 16.0;
  auto key_for = [&](double above) { return R - 1.0 - above * R / N; };   // E #(key > t) = above
  double hi = K - M <= 0.0 ? R - 1.0 : ceil(key_for(K - M));
  double lo = K + M >= N ? 0.0 : floor(key_for(K + M));
  hi = std::min(std::max(hi, 0.0), R - 1.0);
  lo = std::min(std::max(lo, 0.0), hi);
  *t_hi = (uint32_t)hi;
  *t_lo = (uint32_t)lo;
  const uint64_t span = (uint64_t)*t_hi - *t_lo;
  uint32_t sb = 0;
  while ((span >> sb) >= (uint64_t)kHistBins) ++sb;
  *sbin = sb;
}

// k_setup_bracket for one client (jobs == nullptr) or a batch (grid = clients)
static int launch_setup(uint64_t n, uint64_t k, const WsPtrs& W, fc_packet_hdr* hdr,
                        const HdrInit& hi, const fc_encode_job* jobs, uint64_t stride,
                        uint32_t m, hipStream_t s) {
  SetupArgs a;
  memset(&a, 0, sizeof a);
  a.W = W; a.hdr = hdr; a.HI = hi; a.jobs = jobs; a.ws_stride = stride; a.ib = hi.ib;
  philox_bracket(n, k, &a.t_lo, &a.t_hi, &a.sbin);
  TimedLaunch t(FC_TIME_SAMPLE, s);
  hipLaunchKernelGGL(k_setup_bracket, dim3(m), dim3(64), 0, s, a);
  FC_LAUNCHED("k_setup_bracket");
  return FC_OK;
}

// k_fused_mag (sample + compaction in one launch) for a lone magnitude-key client;
// FC_UNFUSED=1 selects the two-launch form in FC_DEBUG_BUILD libraries only (A/B).
static bool fused_enabled() {
#ifdef FC_DEBUG_BUILD
  static const bool on = [] {
    const char* e = getenv("FC_UNFUSED");
    return !(e && atoi(e) != 0);
  }();
  return on;
#else
  return true;
#endif
}

// ---- per-device ordering of the launches whose workgroups wait in-kernel -------------------
// k_fused_mag and k_fused64 hold their compaction workgroups in a bounded poll for the bracket
// their own sample workgroups publish.  Two such launches on two streams are dispatched to the
// XCDs interleaved, so an XCD can fill with waiters whose partners are queued behind another
// full XCD (a stall to the poll bound, then RETRY).  The library itself queues every such launch
// of a device after the previous one: it records its event on the launch's stream after each
// launch and, when the next one comes on another stream, makes that stream wait for the event.
// A stream being captured into a graph is left alone (a replay is ordered by
// fc_fused_order_begin / _end around it).
namespace {
struct FusedOrder {
  std::mutex mu;
  hipEvent_t ev = nullptr;
  hipStream_t last = nullptr;
  bool pending = false;
};
constexpr int kMaxDevices = 64;
FusedOrder g_fused_order[kMaxDevices];

int stream_device(hipStream_t s) {
  int dev = 0;
  if (s == nullptr || hipStreamGetDevice(s, &dev) != hipSuccess) (void)hipGetDevice(&dev);
  return dev & (kMaxDevices - 1);
}

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

class FusedGuard {
 public:
  explicit FusedGuard(hipStream_t s) : s_(s) {
    if (capturing(s)) return;
    const int dev = stream_device(s);
    F_ = &g_fused_order[dev];
    F_->mu.lock();
    if (!F_->ev) {
      int cur = 0;
      (void)hipGetDevice(&cur);
      if (cur != dev) (void)hipSetDevice(dev);
      (void)hipEventCreateWithFlags(&F_->ev, hipEventDisableTiming);
      if (cur != dev) (void)hipSetDevice(cur);
    }
    if (F_->pending && F_->last != s) (void)hipStreamWaitEvent(s, F_->ev, 0);
  }
  // The launch may carry the ordering event itself (hipExtLaunchKernelGGL's stop event: the
  // kernel's own completion signal): a separate hipEventRecord after the kernel put one more
  // packet between consecutive launches, ~3 us per call (profiles/r06_ab_fused_order_event.jsonl).
  hipEvent_t stop_event() const { return F_ ? F_->ev : nullptr; }
  void recorded() { rec_ = true; }
  ~FusedGuard() {
    if (!F_) return;
    if (!rec_) (void)hipEventRecord(F_->ev, s_);
    F_->last = s_;
    F_->pending = true;
    F_->mu.unlock();
  }
  FusedGuard(const FusedGuard&) = delete;
  FusedGuard& operator=(const FusedGuard&) = delete;

 private:
  hipStream_t s_;
  FusedOrder* F_ = nullptr;
  bool rec_ = false;
};
}  // namespace

extern "C" int fc_fused_order_begin(fc_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  FusedOrder& F = g_fused_order[stream_device(s)];
  std::lock_guard<std::mutex> g(F.mu);
  if (F.pending && F.last != s && hipStreamWaitEvent(s, F.ev, 0) != hipSuccess)
    return fail(FC_ERR_HIP, "fc_fused_order_begin: hipStreamWaitEvent");
  return FC_OK;
}

extern "C" int fc_fused_order_end(fc_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  const int dev = stream_device(s);
  FusedOrder& F = g_fused_order[dev];
  std::lock_guard<std::mutex> g(F.mu);
  if (!F.ev) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (cur != dev) (void)hipSetDevice(dev);
    (void)hipEventCreateWithFlags(&F.ev, hipEventDisableTiming);
    if (cur != dev) (void)hipSetDevice(cur);
  }
  if (hipEventRecord(F.ev, s) != hipSuccess) return fail(FC_ERR_HIP, "fc_fused_order_end: hipEventRecord");
  F.last = s;
  F.pending = true;
  return FC_OK;
}

static int launch_fused(const CompactArgs& ca, const SamplePlan& P, const HdrInit& hi,
                         uint32_t nsamp, hipStream_t s) {
  FusedGuard order(s);
  TimedLaunch t(FC_TIME_COMPACT, s);
  const dim3 grid(nsamp + ca.nchunks);
  const hipEvent_t ev = order.stop_event();       // null while capturing: a plain launch
  if (ca.dense) hipExtLaunchKernelGGL(k_fused_mag<true>, grid, dim3(kCBlock), 0, s, nullptr, ev, 0, ca, P, hi, nsamp);
  else hipExtLaunchKernelGGL(k_fused_mag<false>, grid, dim3(kCBlock), 0, s, nullptr, ev, 0, ca, P, hi, nsamp);
  FC_LAUNCHED("k_fused_mag");
  if (ev) order.recorded();
  return FC_OK;
}

// k_resolve workgroups per client: `want`, fewer for a small gradient, more when a workgroup would
// get more than kResolveChunksMax chunks (its LDS size list; with more it reports RETRY: a lone
// encode near n = 2^32, a batch of gradients above 128 M elements)
static uint32_t resolve_grid(uint32_t nchunks, uint32_t want) {
  const uint32_t g = nchunks < want ? nchunks : want;
  const uint32_t need = (nchunks + kResolveChunksMax - 1) / kResolveChunksMax;
  return g > need ? g : need;
}

constexpr int FC_RESOLVE_CPW = 8;          // lone encode: >= this many chunks per k_resolve workgroup
// k_resolve<true> (a.rbin: the compaction left the binning to the resolve) then k_resolve<false>:
// no workgroup of either launch waits for another (only last-arriver tickets), so they are
// safe beside any other kernel, encodes on other streams included
static int launch_resolve(const ResolveArgs& a, hipStream_t s, dim3 grid) {
  TimedLaunch t(FC_TIME_ENGINE, s);
  if (a.rbin) {
    hipLaunchKernelGGL(k_resolve<true>, grid, dim3(kBlock), 0, s, a);
    FC_LAUNCHED("k_resolve<bin>");
  }
  hipLaunchKernelGGL(k_resolve<false>, grid, dim3(kBlock), 0, s, a);
  FC_LAUNCHED("k_resolve<gather>");
  return FC_OK;
}

static int launch_resolve(const ResolveArgs& a, hipStream_t s) {
  const uint32_t want = std::max<uint32_t>(32u, std::min<uint32_t>((uint32_t)kResolveGrid,
                                            (a.nchunks + FC_RESOLVE_CPW - 1) / FC_RESOLVE_CPW));
  return launch_resolve(a, s, dim3(resolve_grid(a.nchunks, want)));
}

extern "C" {

int fc_abi_version(void) { return FC_ABI_VERSION; }
#ifdef FC_TRACE
// diagnostic builds only: copy the phase timestamps (fc_common.h FC_TR) to the host
int fc_trace_read(uint64_t* host, size_t count) {
  if (count > (1u << 16)) count = 1u << 16;
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fc_trace), count * 8, 0, hipMemcpyDeviceToHost);
  return e == hipSuccess ? FC_OK : fail(FC_ERR_HIP, "trace read: %s", hipGetErrorString(e));
}
#endif
const char* fc_last_error(void) { return g_err; }
uint64_t fc_num_chunks(uint64_t n) { return num_chunks(n); }
size_t fc_workspace_bytes(uint64_t n) { return (size_t)WsLayout::of(n).bytes; }
uint64_t fc_packet_capacity(uint64_t n) { return (uint64_t)num_chunks(n) * kChunk; }

int fc_timing_begin(uint32_t mask) {
  g_time_mask = mask;
  g_ev_used = 0;
  return FC_OK;
}

int fc_timing_end(double* total_ms, uint64_t* launches) {
  FC_CHECK(total_ms && launches, "NULL argument");
  for (int c = 0; c < 4; ++c) { total_ms[c] = 0.0; launches[c] = 0; }
  int rc = FC_OK;
  for (size_t i = 0; i < g_ev_used; ++i) {
    float ms = 0.f;
    if (hipEventSynchronize(g_ev[i].b) != hipSuccess ||
        hipEventElapsedTime(&ms, g_ev[i].a, g_ev[i].b) != hipSuccess) {
      rc = fail(FC_ERR_HIP, "timing events failed");
      continue;
    }
    const int c = __builtin_ctz(g_ev[i].cat);
    total_ms[c] += ms;
    launches[c] += 1;
  }
  g_time_mask = 0;
  g_ev_used = 0;
  return rc;
}

int fc_workspace_init(void* ws, size_t ws_bytes, fc_stream_t stream) {
  FC_CHECK(ws != nullptr, "workspace is NULL");
  hipError_t e = hipMemsetAsync(ws, 0, ws_bytes, (hipStream_t)stream);
  if (e != hipSuccess) return fail(FC_ERR_HIP, "hipMemsetAsync: %s", hipGetErrorString(e));
  return FC_OK;
}

static int topk_args(const float* g, uint64_t n, uint64_t k, int key_mode, uint64_t seed,
                     uint64_t offset, uint16_t* idx, float* val, uint64_t capacity,
                     uint32_t* cnt, uint64_t* qoff, fc_packet_hdr* hdr, void* ws,
                     size_t ws_bytes, CompactArgs* ca, EngineArgs* ea, ResolveArgs* ra,
                     HdrInit* hi) {
  int rc = check_common(g, n, ws, ws_bytes);
  if (rc) return rc;
  FC_CHECK(idx && val && cnt && hdr, "packet buffers must be non-NULL");
  FC_CHECK(key_mode == FC_KEY_MAGNITUDE || key_mode == FC_KEY_PHILOX, "bad key_mode %d", key_mode);
  FC_CHECK(k <= n, "k=%llu > n=%llu (pass the effective k)", (unsigned long long)k,
           (unsigned long long)n);
  FC_CHECK(capacity >= fc_packet_capacity(n), "capacity %llu < fc_packet_capacity(n) %llu",
           (unsigned long long)capacity, (unsigned long long)fc_packet_capacity(n));
  const uint32_t ib = index_bits(n);
  memset(hi, 0, sizeof *hi);
  hi->seed = seed; hi->offset = offset; hi->p = 0.0; hi->n = (uint32_t)n; hi->k = (uint32_t)k;
  hi->ib = ib; hi->codec = key_mode == FC_KEY_PHILOX ? FC_CODEC_RAND : FC_CODEC_TOP;
  hi->format = FC_FMT_IDXVAL; hi->key_mode = (uint32_t)key_mode;
  memset(ca, 0, sizeof *ca);
  ca->g = g; ca->n = n; ca->ib = ib; ca->nchunks = num_chunks(n);
  ca->seed = seed; ca->offset = offset; ca->idx = idx; ca->val = val; ca->cnt = cnt;
  ca->qoff = qoff;
  ca->hdr = hdr; ca->W = ws_ptrs(ws, n); ca->HI = *hi;
  memset(ea, 0, sizeof *ea);
  ea->g = g; ea->n = n; ea->ib = ib; ea->k = k;
  ea->seed = seed; ea->offset = offset; ea->hdr = hdr; ea->W = ca->W; ea->HI = *hi;
  memset(ra, 0, sizeof *ra);
  ra->ib = ib; ra->nchunks = ca->nchunks; ra->k = k; ra->idx = idx; ra->val = val; ra->cnt = cnt;
  ra->seed = seed; ra->offset = offset; ra->key_mode = (uint32_t)key_mode;
  ra->hdr = hdr; ra->W = ca->W;
  return FC_OK;
}

int fc_topk_encode_exact(const float* g, uint64_t n, uint64_t k, int key_mode, uint64_t seed,
                         uint64_t offset, uint16_t* idx, float* val, uint64_t capacity,
                         uint32_t* cnt, uint64_t* qoff, fc_packet_hdr* hdr, void* ws,
                         size_t ws_bytes, fc_stream_t stream) {
  CompactArgs ca; EngineArgs ea; ResolveArgs ra; HdrInit hi;
  int rc = topk_args(g, n, k, key_mode, seed, offset, idx, val, capacity, cnt, qoff, hdr, ws,
                     ws_bytes, &ca, &ea, &ra, &hi);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  rc = launch_engine(key_mode, ea, kEnginePasses, s);
  if (rc) return rc;
  return launch_compact_key(key_mode, ca, s);
}

int fc_topk_encode(const float* g, uint64_t n, uint64_t k, int key_mode, uint64_t seed,
                   uint64_t offset, uint16_t* idx, float* val, uint64_t capacity,
                   uint32_t* cnt, uint64_t* qoff, fc_packet_hdr* hdr, void* ws,
                   size_t ws_bytes, fc_stream_t stream) {
  if (k == 0 || k >= n)  // trivial thresholds: the exact engine resolves them in its init
    return fc_topk_encode_exact(g, n, k, key_mode, seed, offset, idx, val, capacity, cnt, qoff,
                                hdr, ws, ws_bytes, stream);
  CompactArgs ca; EngineArgs ea; ResolveArgs ra; HdrInit hi;
  int rc = topk_args(g, n, k, key_mode, seed, offset, idx, val, capacity, cnt, qoff, hdr, ws,
                     ws_bytes, &ca, &ea, &ra, &hi);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const SamplePlan P = make_plan(n, k);
  const uint32_t sgrid = (P.nseg + P.segs - 1) / P.segs;   // <= 256
  if (key_mode == FC_KEY_MAGNITUDE && fused_enabled()) {
    rc = launch_fused(ca, P, hi, sgrid, s);
    if (rc) return rc;
    ra.rbin = 0;                     // k_fused_mag binned the candidates
    return launch_resolve(ra, s);
  }
  if (key_mode == FC_KEY_PHILOX)      // uniform keys: the analytical bracket, no sample
    rc = launch_setup(n, k, ca.W, hdr, hi, nullptr, 0ull, 1, s);
  else
    rc = launch_sample(key_mode, dim3(sgrid), g, P, seed, offset, ca.W, ca.ib, hdr, hi, nullptr, 0ull, s);
  if (rc) return rc;
  const bool bin = key_mode == FC_KEY_PHILOX;   // rand-k bins its candidates while it compacts
  rc = launch_compact_key(key_mode, ca, s, 1, bin);
  if (rc) return rc;
  ra.rbin = bin ? 0 : 1;             // else the unfused compaction leaves the binning to k_resolve
  return launch_resolve(ra, s);
}

int fc_topk_encode_decode(const float* g, uint64_t n, uint64_t k, uint16_t* idx, float* val,
                          uint64_t capacity, uint32_t* cnt, uint64_t* qoff, fc_packet_hdr* hdr,
                          void* ws, size_t ws_bytes, float* out, fc_stream_t stream) {
  FC_CHECK(k > 0 && k < n, "fc_topk_encode_decode needs 0 < k < n (k=%llu, n=%llu)",
           (unsigned long long)k, (unsigned long long)n);
  FC_CHECK(qoff != nullptr, "fc_topk_encode_decode needs the quarter offsets (qoff)");
  FC_CHECK(out != nullptr && ((uintptr_t)out & 15) == 0, "out must be non-NULL and 16-byte aligned");
  CompactArgs ca; EngineArgs ea; ResolveArgs ra; HdrInit hi;
  int rc = topk_args(g, n, k, FC_KEY_MAGNITUDE, 0, 0, idx, val, capacity, cnt, qoff, hdr, ws,
                     ws_bytes, &ca, &ea, &ra, &hi);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const SamplePlan P = make_plan(n, k);
  const uint32_t sgrid = (P.nseg + P.segs - 1) / P.segs;
  // the packet, exactly fc_topk_encode's; then the bin beta in one workgroup (as the fused
  // launch's own tail — a last-arriver ticket in every chunk workgroup — it cost more than this
  // launch: 128 M 141.4 -> 147.1 us, 16 M 35.5 -> 43.5 us, profiles/r06_lone_probe.jsonl)
  rc = launch_fused(ca, P, hi, sgrid, s);
  if (rc) return rc;
  {
    TimedLaunch t(FC_TIME_ENGINE, s);
    hipLaunchKernelGGL(k_beta, dim3(1), dim3(kBlock), 0, s, ra);
    FC_LAUNCHED("k_beta");
  }
  DecResArgs d;
  memset(&d, 0, sizeof d);
  d.idx = idx; d.val = val; d.qoff = qoff; d.hdr = hdr; d.out = out; d.n = n;
  d.ib = index_bits(n); d.W = ws_ptrs(ws, n);
  TimedLaunch t(FC_TIME_DECODE, s);
  hipLaunchKernelGGL(k_decode_res, dim3(num_chunks(n)), dim3(kQBlock), 0, s, d);
  FC_LAUNCHED("k_decode_res");
  return FC_OK;
}

int fc_topk_encode_dense(const float* g, uint64_t n, uint64_t k, uint16_t* idx, float* val,
                         uint64_t capacity, uint32_t* cnt, uint64_t* qoff, fc_packet_hdr* hdr,
                         void* ws, size_t ws_bytes, float* dense, fc_stream_t stream) {
  FC_CHECK(dense != nullptr, "dense is NULL");
  FC_CHECK(((uintptr_t)dense & 15) == 0, "dense must be 16-byte aligned");
  FC_CHECK(k > 0 && k < n, "fc_topk_encode_dense needs 0 < k < n (trivial k: encode + decode)");
  CompactArgs ca; EngineArgs ea; ResolveArgs ra; HdrInit hi;
  int rc = topk_args(g, n, k, FC_KEY_MAGNITUDE, 0, 0, idx, val, capacity, cnt, qoff, hdr, ws,
                     ws_bytes, &ca, &ea, &ra, &hi);
  if (rc) return rc;
  ca.dense = dense;
  if (fused_enabled()) {             // q is the product: the header says no entries
    hi.format = FC_FMT_DENSE;
    ca.HI.format = FC_FMT_DENSE;
  }
  hipStream_t s = (hipStream_t)stream;
  const SamplePlan P = make_plan(n, k, true);
  const uint32_t sgrid = (P.nseg + P.segs - 1) / P.segs;
  if (fused_enabled()) {
    rc = launch_fused(ca, P, hi, sgrid, s);
    if (rc) return rc;
    ra.rbin = 0;                     // k_fused_mag binned the candidates
  } else {
    ra.rbin = 1;
    rc = launch_sample(FC_KEY_MAGNITUDE, dim3(sgrid), g, P, 0ull, 0ull, ca.W, ca.ib, hdr, hi, nullptr, 0ull, s);
    if (rc) return rc;
    TimedLaunch t(FC_TIME_COMPACT, s);
    const dim3 grid = compact_mag_grid(ca, 1);
    hipLaunchKernelGGL(k_compact_mag1_dense, grid, dim3(kCBlock), 0, s, ca);
    FC_LAUNCHED("k_compact_mag1_dense");
  }
  // k_resolve publishes T64 to its own workgroups, which then zero the slack in q
  ra.dense = dense;
  return launch_resolve(ra, s);
}

size_t fc_workspace_bytes_batch(uint64_t n, int m) {
  return m > 0 ? (size_t)WsLayout::of(n).bytes * (size_t)m : 0;
}

int fc_topk_encode_batch(const fc_encode_job* jobs, int m, uint64_t n, uint64_t k,
                         int key_mode, uint64_t capacity, void* ws, size_t ws_bytes,
                         fc_stream_t stream) {
  return fc_topk_encode_batch_part(jobs, m, n, k, key_mode, capacity, ws, ws_bytes,
                                   FC_PART_SAMPLE | FC_PART_FINISH, stream);
}

int fc_topk_encode_batch_part(const fc_encode_job* jobs, int m, uint64_t n, uint64_t k,
                              int key_mode, uint64_t capacity, void* ws, size_t ws_bytes,
                              int part, fc_stream_t stream) {
  FC_CHECK(part >= 1 && part <= (FC_PART_SAMPLE | FC_PART_FINISH), "bad part %d", part);
  FC_CHECK(jobs != nullptr, "jobs is NULL");
  FC_CHECK(m >= 1 && m <= 65535, "m=%d outside [1, 65535]", m);
  FC_CHECK(n >= 2 && n <= 0xffffffffull, "n=%llu outside [2, 2^32-1]", (unsigned long long)n);
  FC_CHECK(k > 0 && k < n, "batched encode needs 0 < k < n (k=%llu): use fc_topk_encode",
           (unsigned long long)k);
  FC_CHECK(key_mode == FC_KEY_MAGNITUDE || key_mode == FC_KEY_PHILOX, "bad key_mode %d", key_mode);
  FC_CHECK(capacity >= fc_packet_capacity(n), "capacity %llu < fc_packet_capacity(n) %llu",
           (unsigned long long)capacity, (unsigned long long)fc_packet_capacity(n));
  FC_CHECK(ws != nullptr, "workspace is NULL");
  if (ws_bytes < fc_workspace_bytes_batch(n, m))
    return fail(FC_ERR_WORKSPACE, "workspace %zu B < %zu B needed", ws_bytes,
                fc_workspace_bytes_batch(n, m));
  const uint32_t ib = index_bits(n);
  const uint64_t stride = WsLayout::of(n).bytes;
  HdrInit hi;
  memset(&hi, 0, sizeof hi);
  hi.n = (uint32_t)n; hi.k = (uint32_t)k; hi.ib = ib;
  hi.codec = key_mode == FC_KEY_PHILOX ? FC_CODEC_RAND : FC_CODEC_TOP;
  hi.format = FC_FMT_IDXVAL; hi.key_mode = (uint32_t)key_mode;
  CompactArgs ca;
  memset(&ca, 0, sizeof ca);
  ca.n = n; ca.ib = ib; ca.nchunks = num_chunks(n); ca.W = ws_ptrs(ws, n); ca.HI = hi;
  ca.jobs = jobs; ca.ws_stride = stride;
  ResolveArgs ra;
  memset(&ra, 0, sizeof ra);
  ra.ib = ib; ra.nchunks = ca.nchunks; ra.k = k; ra.key_mode = (uint32_t)key_mode;
  ra.W = ca.W; ra.jobs = jobs; ra.ws_stride = stride;
  ra.rbin = 1;                       // batched compaction: k_resolve bins the candidates
  hipStream_t s = (hipStream_t)stream;
  SamplePlan P = make_plan(n, k);
  P.cbins_log2 = cand_bins_log2(n, P);
  // FC_SAMPLE_ROUNDS sample groups per workgroup (k_sample1): the same sample, fewer workgroups
  const dim3 sgrid((P.pstride + FC_SAMPLE_ROUNDS - 1) / FC_SAMPLE_ROUNDS, (uint32_t)m);
  if (part & FC_PART_SAMPLE) {
    int rc = key_mode == FC_KEY_PHILOX
                 ? launch_setup(n, k, ca.W, nullptr, hi, jobs, stride, (uint32_t)m, s)
                 : launch_sample(key_mode, sgrid, nullptr, P, 0ull, 0ull, ca.W, ib, nullptr, hi, jobs, stride, s);
    if (rc) return rc;
  }
  if (!(part & FC_PART_FINISH)) return FC_OK;
  {
    int rc = launch_compact_key(key_mode, ca, s, (uint32_t)m);
    if (rc) return rc;
  }
  // fewer resolve workgroups per client than a lone encode: the batch fills the chip
  return launch_resolve(ra, s, dim3(resolve_grid(ca.nchunks, kResolveGridBatch), (uint32_t)m));
}

int fc_mask_encode(const float* g, uint64_t n, int codec, const uint32_t* mask_bits, double p,
                   uint64_t seed, uint64_t offset, int format, uint16_t* idx, float* val,
                   uint32_t* bitmap, uint64_t capacity, uint32_t* cnt, uint64_t* qoff,
                   fc_packet_hdr* hdr, void* ws, size_t ws_bytes, fc_stream_t stream) {
  int rc = check_common(g, n, ws, ws_bytes);
  if (rc) return rc;
  FC_CHECK(codec == FC_CODEC_DROPOUT_BIASED || codec == FC_CODEC_DROPOUT_UNBIASED ||
               codec == FC_CODEC_RAND, "bad codec %d", codec);
  FC_CHECK(format == FC_FMT_IDXVAL || format == FC_FMT_BITMAP, "bad format %d", format);
  FC_CHECK(val && cnt && hdr, "packet buffers must be non-NULL");
  FC_CHECK(format != FC_FMT_IDXVAL || idx, "idx required for FC_FMT_IDXVAL");
  FC_CHECK(format != FC_FMT_BITMAP || bitmap, "bitmap required for FC_FMT_BITMAP");
  FC_CHECK(capacity >= fc_packet_capacity(n), "capacity %llu < fc_packet_capacity(n) %llu",
           (unsigned long long)capacity, (unsigned long long)fc_packet_capacity(n));
  FC_CHECK(mask_bits || (p >= 0.0 && p <= 1.0), "p=%g outside [0, 1]", p);
  FC_CHECK(mask_bits || codec != FC_CODEC_RAND, "native rand-k uses fc_topk_encode(PHILOX)");
  HdrInit hi;
  memset(&hi, 0, sizeof hi);
  hi.seed = seed; hi.offset = offset; hi.p = p; hi.n = (uint32_t)n; hi.k = 0;
  hi.ib = index_bits(n); hi.codec = (uint32_t)codec; hi.format = (uint32_t)format;
  hi.key_mode = FC_KEY_MAGNITUDE;
  CompactArgs a;
  memset(&a, 0, sizeof a);
  a.g = g; a.n = n; a.ib = hi.ib; a.nchunks = num_chunks(n);
  a.seed = seed; a.offset = offset; a.mask = mask_bits;
  double thr = floor(p * 4294967296.0 + 0.5);
  if (thr < 0) thr = 0;
  if (thr > 4294967296.0) thr = 4294967296.0;
  a.bern_thr = (uint64_t)thr;
  a.nonfinite_keep = codec != FC_CODEC_RAND;
  a.write_hdr = 1; a.idx = idx; a.val = val; a.bitmap = bitmap; a.cnt = cnt;
  a.qoff = format == FC_FMT_IDXVAL ? qoff : nullptr;
  a.hdr = hdr; a.W = ws_ptrs(ws, n); a.HI = hi;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(a.nchunks), blk(kCBlock);
  const PredArgs pa = pred_args(a);
  {
    TimedLaunch t(FC_TIME_COMPACT, s);
    if (mask_bits) {
      if (format == FC_FMT_BITMAP) hipLaunchKernelGGL((k_compact_pred<kSrcMaskBits, FC_FMT_BITMAP>), grid, blk, 0, s, pa);
      else hipLaunchKernelGGL((k_compact_pred<kSrcMaskBits, FC_FMT_IDXVAL>), grid, blk, 0, s, pa);
    } else {
      if (format == FC_FMT_BITMAP) hipLaunchKernelGGL((k_compact_pred<kSrcBern, FC_FMT_BITMAP>), grid, blk, 0, s, pa);
      else hipLaunchKernelGGL((k_compact_pred<kSrcBern, FC_FMT_IDXVAL>), grid, blk, 0, s, pa);
    }
    FC_LAUNCHED("k_compact_pred(mask)");
  }
  // the packet's static header (its only writer; decoders read it after this stream point)
  hipLaunchKernelGGL(k_write_hdr, dim3(1), dim3(64), 0, s, hdr, hi);
  FC_LAUNCHED("k_write_hdr");
  return FC_OK;
}

int fc_decode_dense(const fc_packet_view* pkt, int format, uint64_t n, void* out, int out_f64,
                    fc_stream_t stream) {
  FC_CHECK(pkt && out, "NULL argument");
  FC_CHECK(n >= 1 && n <= 0xffffffffull, "bad n");
  FC_CHECK(format == FC_FMT_IDXVAL || format == FC_FMT_BITMAP, "bad format %d", format);
  FC_CHECK(pkt->cnt && pkt->hdr && pkt->val, "packet view incomplete");
  FC_CHECK(format != FC_FMT_IDXVAL || pkt->idx, "idx missing");
  FC_CHECK(format != FC_FMT_BITMAP || pkt->bitmap, "bitmap missing");
  FC_CHECK(((uintptr_t)out & 15) == 0, "out must be 16-byte aligned");
  DecodeArgs a;
  memset(&a, 0, sizeof a);
  a.views = nullptr; a.one = *pkt; a.m = 1; a.n = n; a.out = out;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(decode_grid(n)), blk(kDBlock);
  TimedLaunch t(FC_TIME_DECODE, s);
  if (format == FC_FMT_IDXVAL) {
    if (out_f64) hipLaunchKernelGGL((k_decode<FC_FMT_IDXVAL, false, true>), grid, blk, 0, s, a);
    // dense decode: 4 resident WGs per CU (no fold counters in LDS); 1024 WGs measured 3 %
    // faster than 768 and 14 % faster than one WG per chunk
    // dense decode: the quarter-owned waves of the fold (no barrier per chunk): 87.5 us at
    // 128 M against 109.5 for k_decode_sparse<false> and its per-chunk workgroup barriers
    // (at 16 M the barrier form is 0.5 us faster: 2048 one-chunk workgroups in ~2 rounds)
    else if (num_chunks(n) >= 4096u)
      hipLaunchKernelGGL((k_fold_q<false, true>), dim3(num_chunks(n)), dim3(kQBlock), 0, s, a);
    else hipLaunchKernelGGL(k_decode_sparse<false>, dim3(decode_grid(n, 4)), dim3(kSBlock), 0, s, a);
  } else {
    if (out_f64) hipLaunchKernelGGL((k_decode<FC_FMT_BITMAP, false, true>), grid, blk, 0, s, a);
    else hipLaunchKernelGGL((k_decode<FC_FMT_BITMAP, false, false>), grid, blk, 0, s, a);
  }
  FC_LAUNCHED("k_decode");
  return FC_OK;
}

static int decode_accumulate(const fc_packet_view* views_dev, int m, int format, uint64_t n,
                             float* acc, bool cont, fc_stream_t stream) {
  FC_CHECK(views_dev && acc, "NULL argument");
  FC_CHECK(m >= 1, "m=%d < 1", m);
  FC_CHECK(n >= 1 && n <= 0xffffffffull, "bad n");
  FC_CHECK(format == FC_FMT_IDXVAL || format == FC_FMT_BITMAP, "bad format %d", format);
  FC_CHECK(((uintptr_t)acc & 15) == 0, "acc must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(decode_grid(n)), blk(kDBlock);
  // <= kSparseMaxM (idx/val) or kDecMaxM (bitmap) packets per launch; later launches
  // continue the same left-to-right sum
  const int per_launch = format == FC_FMT_IDXVAL ? kSparseMaxM : kDecMaxM;
  for (int m0 = 0; m0 < m; m0 += per_launch) {
    DecodeArgs a;
    memset(&a, 0, sizeof a);
    a.views = views_dev + m0; a.m = std::min(m - m0, per_launch); a.acc_in = cont || m0 > 0;
    a.n = n; a.out = acc;
    TimedLaunch t(FC_TIME_DECODE, s);
    if (format == FC_FMT_IDXVAL) {
      // fold: one workgroup per chunk, each wave folding its own quarter (no barriers)
      if (a.acc_in) hipLaunchKernelGGL(k_fold_q<true>, dim3(num_chunks(n)), dim3(kQBlock), 0, s, a);
      else hipLaunchKernelGGL(k_fold_q<false>, dim3(num_chunks(n)), dim3(kQBlock), 0, s, a);
    } else {
      hipLaunchKernelGGL((k_decode<FC_FMT_BITMAP, true, false>), grid, blk, 0, s, a);
    }
    FC_LAUNCHED("k_decode(acc)");
  }
  return FC_OK;
}

int fc_decode_accumulate(const fc_packet_view* views_dev, int m, int format, uint64_t n,
                         float* acc, fc_stream_t stream) {
  return decode_accumulate(views_dev, m, format, n, acc, false, stream);
}

int fc_decode_accumulate_continue(const fc_packet_view* views_dev, int m, int format,
                                  uint64_t n, float* acc, fc_stream_t stream) {
  return decode_accumulate(views_dev, m, format, n, acc, true, stream);
}

uint64_t fc_qsgd_code_words(uint64_t n, int bits) {
  if (bits < 1 || bits > 14) return 0;
  return (n + kQsgdElems - 1) / kQsgdElems * (uint64_t)(qsgd_width(bits) * kQsgdElems / 32);
}
size_t fc_qsgd_workspace_bytes(void) { return 64 + 8 * (size_t)kQsgdNormGrid; }

// Grid caps of the QSGD passes (grid-stride loops): quantise 8192 workgroups (113 us per 128 M,
// 4096: 116, 1024: 138), lone decode 1024 (99 us, 4096: 111), fold one lane tile per thread.
constexpr int FC_QSGD_QGRID = 8192;
constexpr int FC_QSGD_DGRID = 1024;
constexpr int FC_QSGD_FGRID = 65535;
static uint32_t stream_grid(uint64_t items, uint64_t cap) {
  uint64_t b = (items + kBlock - 1) / kBlock;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (uint32_t)b;
}

int fc_qsgd_encode(const float* g, uint64_t n, int bits, uint64_t seed, uint64_t offset,
                   uint32_t* codes, uint64_t code_words, fc_packet_hdr* hdr, void* ws,
                   size_t ws_bytes, fc_stream_t stream) {
  FC_CHECK(g && codes && hdr && ws, "NULL argument");
  FC_CHECK(n >= 1 && n <= 0xffffffffull, "n=%llu outside [1, 2^32-1]", (unsigned long long)n);
  FC_CHECK(bits >= 1 && bits <= 14, "bits=%d outside [1, 14]", bits);
  FC_CHECK(((uintptr_t)g & 15) == 0 && ((uintptr_t)codes & 15) == 0, "g and codes must be 16-byte aligned");
  FC_CHECK(code_words >= fc_qsgd_code_words(n, bits), "code_words %llu < %llu needed",
           (unsigned long long)code_words, (unsigned long long)fc_qsgd_code_words(n, bits));
  if (ws_bytes < fc_qsgd_workspace_bytes())
    return fail(FC_ERR_WORKSPACE, "workspace %zu B < %zu B needed", ws_bytes, fc_qsgd_workspace_bytes());
  hipStream_t s = (hipStream_t)stream;
  char* w = static_cast<char*>(ws);
  uint64_t ng = (n / 4 + kBlock - 1) / kBlock;                 // fixed for a given n
  if (ng < 1) ng = 1;
  if (ng > (uint64_t)kQsgdNormGrid) ng = kQsgdNormGrid;
  {
    TimedLaunch t(FC_TIME_SAMPLE, s);
    hipLaunchKernelGGL(k_qsgd_norm, dim3((uint32_t)ng), dim3(kBlock), 0, s, g, n, bits, seed, offset,
                       reinterpret_cast<double*>(w + 64), reinterpret_cast<uint32_t*>(w), hdr);
    FC_LAUNCHED("k_qsgd_norm");
  }
  TimedLaunch t(FC_TIME_COMPACT, s);
  hipLaunchKernelGGL(k_qsgd_quant, dim3(stream_grid((n + kQsgdElems - 1) / kQsgdElems, FC_QSGD_QGRID)), dim3(kBlock), 0, s,
                     g, n, bits, seed, offset, hdr, codes);
  FC_LAUNCHED("k_qsgd_quant");
  return FC_OK;
}

int fc_qsgd_decode(const fc_packet_view* pkt, uint64_t n, float* out, fc_stream_t stream) {
  FC_CHECK(pkt && out && pkt->idx && pkt->hdr, "NULL argument");
  FC_CHECK(n >= 1 && n <= 0xffffffffull, "bad n");
  FC_CHECK(((uintptr_t)out & 15) == 0 && ((uintptr_t)pkt->idx & 15) == 0, "out and codes must be 16-byte aligned");
  QsgdDecodeArgs a;
  memset(&a, 0, sizeof a);
  a.one = *pkt; a.m = 1; a.n = n; a.out = out;
  hipStream_t s = (hipStream_t)stream;
  TimedLaunch t(FC_TIME_DECODE, s);
  hipLaunchKernelGGL(k_qsgd_decode<false>, dim3(stream_grid((n + 3) / 4, FC_QSGD_DGRID)), dim3(kBlock), 0, s, a);
  FC_LAUNCHED("k_qsgd_decode");
  return FC_OK;
}

int fc_qsgd_decode_accumulate(const fc_packet_view* views_dev, int m, uint64_t n, float* out,
                              int continue_sum, fc_stream_t stream) {
  FC_CHECK(views_dev && out, "NULL argument");
  FC_CHECK(m >= 1, "m=%d < 1", m);
  FC_CHECK(n >= 1 && n <= 0xffffffffull, "bad n");
  FC_CHECK(((uintptr_t)out & 15) == 0, "out must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  TimedLaunch t(FC_TIME_DECODE, s);
  // kQsgdFoldM packets per launch (their parameters live in LDS); a longer fold continues the
  // previous launch's partial sum in row order (the same additions as one launch)
  for (int m0 = 0; m0 < m; m0 += kQsgdFoldM) {
    QsgdDecodeArgs a;
    memset(&a, 0, sizeof a);
    a.views = views_dev + m0; a.m = std::min(kQsgdFoldM, m - m0);
    a.acc_in = (m0 > 0 || continue_sum != 0) ? 1 : 0; a.n = n; a.out = out;
    hipLaunchKernelGGL(k_qsgd_decode<true>, dim3(stream_grid((n + 31) / 32, FC_QSGD_FGRID)), dim3(kBlock), 0, s, a);
    FC_LAUNCHED("k_qsgd_decode(acc)");
  }
  return FC_OK;
}

int fc_flat_stage(const float* const* params_dev, const uint64_t* offsets_dev, int count,
                  uint64_t max_size, float* flat, float* grad, int scatter, fc_stream_t stream) {
  FC_CHECK(params_dev && offsets_dev && flat, "NULL argument");
  FC_CHECK(count >= 1 && count <= 65535, "count=%d outside [1, 65535]", count);
  FC_CHECK(!(scatter && grad), "scatter takes no grad");
  uint64_t bx = (max_size + kBlock - 1) / kBlock;
  if (bx < 1) bx = 1;
  if (bx > 1024) bx = 1024;
  hipLaunchKernelGGL(k_flat_stage, dim3((uint32_t)bx, (uint32_t)count), dim3(kBlock), 0,
                     (hipStream_t)stream, params_dev, offsets_dev, flat, grad, scatter);
  FC_LAUNCHED("k_flat_stage");
  return FC_OK;
}

int fc_div_scalar(float* x, uint64_t n, float d, fc_stream_t stream) {
  FC_CHECK(x != nullptr, "x is NULL");
  FC_CHECK(n >= 1, "n=0");
  FC_CHECK(((uintptr_t)x & 15) == 0, "x must be 16-byte aligned");
  uint64_t blocks = (n / 4 + kBlock - 1) / kBlock;
  if (blocks < 1) blocks = 1;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(k_div_scalar, dim3((uint32_t)blocks), dim3(kBlock), 0, (hipStream_t)stream,
                     x, n, d);
  FC_LAUNCHED("k_div_scalar");
  return FC_OK;
}

static int weighted_sum_dense(const float* const* rows, const float* w, int m, uint64_t n,
                              float* out, int acc_in, fc_stream_t stream) {
  FC_CHECK(rows && w && out, "NULL argument");
  FC_CHECK(m >= 1, "m=%d < 1", m);
  FC_CHECK(n >= 1, "n=0");
  FC_CHECK(((uintptr_t)out & 15) == 0, "out must be 16-byte aligned");
  const uint64_t nq = (n + 3) / 4;
  uint64_t blocks = (nq + kBlock - 1) / kBlock;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(k_wsum, dim3((uint32_t)blocks), dim3(kBlock), 0, (hipStream_t)stream, rows,
                     w, m, n, out, acc_in);
  FC_LAUNCHED("k_wsum");
  return FC_OK;
}

int fc_weighted_sum_dense(const float* const* rows, const float* w, int m, uint64_t n,
                          float* out, fc_stream_t stream) {
  return weighted_sum_dense(rows, w, m, n, out, 0, stream);
}

int fc_weighted_sum_dense_continue(const float* const* rows, const float* w, int m, uint64_t n,
                                   float* out, fc_stream_t stream) {
  return weighted_sum_dense(rows, w, m, n, out, 1, stream);
}

// ---- float64 gradients (attack_models.py:105-106 -> aggregation.py:61) -------------------
static uint32_t grid_of(uint64_t n) {
  uint64_t b = (n + kBlock - 1) / kBlock;
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;
  return (uint32_t)b;
}

int fc_topk_dense_f64_sampled(const double* g, uint64_t n, uint64_t k, double* out, void* ws,
                              size_t ws_bytes, uint32_t* status, fc_stream_t stream) {
  FC_CHECK(g && out && ws && status, "NULL argument");
  FC_CHECK(n >= 2 && n <= 0xffffffffull, "n=%llu outside [2, 2^32-1]", (unsigned long long)n);
  FC_CHECK(k > 0 && k < n, "the sampled fp64 path needs 0 < k < n (k=%llu, n=%llu)",
           (unsigned long long)k, (unsigned long long)n);
  FC_CHECK(((uintptr_t)g & 15) == 0 && ((uintptr_t)out & 15) == 0, "g and out must be 16-B aligned");
  const WsLayout Lw = WsLayout::of(n);
  if (ws_bytes < Lw.bytes)
    return fail(FC_ERR_WORKSPACE, "workspace %zu B < %llu B needed", ws_bytes,
                (unsigned long long)Lw.bytes);
  const WsPtrs W = ws_ptrs(ws, n);
  hipStream_t s = (hipStream_t)stream;
  const SamplePlan P = make_plan(n, k, true);
  const uint32_t ib = index_bits(n);
  HdrInit hi;
  memset(&hi, 0, sizeof hi);
  hi.n = (uint32_t)n; hi.k = (uint32_t)k; hi.ib = ib; hi.codec = FC_CODEC_TOP;
  hi.format = FC_FMT_DENSE; hi.key_mode = FC_KEY_MAGNITUDE;
  auto* hdr = reinterpret_cast<fc_packet_hdr*>(static_cast<char*>(ws) + kHdr64Off);
  Fast64Args a;
  memset(&a, 0, sizeof a);
  a.g = g; a.n = n; a.k = k; a.nchunks = (uint32_t)Lw.nchunks;
  // chunks per k_resolve64 workgroup: >= 16, and <= kResolve64Grid workgroups (they wait for
  // each other's T in-kernel)
  a.per = (uint32_t)std::max<uint64_t>(16, (Lw.nchunks + kResolve64Grid - 1) / kResolve64Grid);
  a.S = W.st; a.E = reinterpret_cast<Eng64State*>(static_cast<char*>(ws) + kEng64Off);
  a.ccnt = W.ccnt; a.cand = reinterpret_cast<u128*>(W.cand); a.chist = W.chist;
  a.tick = W.tick + 2 * kTickWords; a.small = reinterpret_cast<u128*>(W.small);
  a.out = out; a.status = status;
  const uint32_t rgrid = (a.nchunks + a.per - 1) / a.per;
  {
    TimedLaunch t(FC_TIME_COMPACT, s);
    const uint32_t nsamp = (P.nseg + P.segs - 1) / P.segs;
    FusedGuard order(s);
    const hipEvent_t ev = order.stop_event();
    hipExtLaunchKernelGGL(k_fused64, dim3(nsamp + a.nchunks), dim3(kBlock), 0, s, nullptr, ev, 0, a, P, W, ib, hdr, hi, nsamp);
    FC_LAUNCHED("k_fused64");
    if (ev) order.recorded();
  }
  {
    TimedLaunch t(FC_TIME_ENGINE, s);
    hipLaunchKernelGGL(k_resolve64, dim3(rgrid), dim3(kBlock), 0, s, a);
    FC_LAUNCHED("k_resolve64");
  }
  return FC_OK;
}

int fc_topk_dense_f64(const double* g, uint64_t n, uint64_t k, int key_mode, uint64_t seed,
                      uint64_t offset, double* out, void* ws, size_t ws_bytes,
                      fc_stream_t stream) {
  FC_CHECK(g && out && ws, "NULL argument");
  FC_CHECK(n >= 1 && n <= 0xffffffffull, "n=%llu outside [1, 2^32-1]", (unsigned long long)n);
  FC_CHECK(k <= n, "k=%llu > n=%llu (pass the effective k)", (unsigned long long)k,
           (unsigned long long)n);
  FC_CHECK(key_mode == FC_KEY_MAGNITUDE || key_mode == FC_KEY_PHILOX, "bad key_mode %d", key_mode);
  if (ws_bytes < WsLayout::of(n).bytes)
    return fail(FC_ERR_WORKSPACE, "workspace %zu B < %llu B needed", ws_bytes,
                (unsigned long long)WsLayout::of(n).bytes);
  const WsPtrs W = ws_ptrs(ws, n);
  Engine64Args a;
  memset(&a, 0, sizeof a);
  a.g = g; a.n = n; a.k = k; a.seed = seed; a.offset = offset; a.key_mode = (uint32_t)key_mode;
  a.E = reinterpret_cast<Eng64State*>(static_cast<char*>(ws) + kEng64Off);
  a.hist = W.ehist;
  a.small = reinterpret_cast<u128*>(W.small);
  hipStream_t s = (hipStream_t)stream;
  for (int p = 0; p < 8; ++p) {                  // 95-bit comps, 12-bit digits: <= 8 passes
    TimedLaunch t(FC_TIME_ENGINE, s);
    a.first = p == 0;
    if (key_mode == FC_KEY_PHILOX) hipLaunchKernelGGL(k_engine64<kKeyPhilox>, dim3(kEngineGrid), dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL(k_engine64<kKeyMag>, dim3(kEngineGrid), dim3(kBlock), 0, s, a);
    FC_LAUNCHED("k_engine64");
  }
  TimedLaunch t(FC_TIME_COMPACT, s);
  if (key_mode == FC_KEY_PHILOX)
    hipLaunchKernelGGL(k_select_dense64<kKeyPhilox>, dim3(grid_of(n)), dim3(kBlock), 0, s, g, n, k, seed, offset, a.E, out);
  else
    hipLaunchKernelGGL(k_select_dense64<kKeyMag>, dim3(grid_of(n)), dim3(kBlock), 0, s, g, n, k, seed, offset, a.E, out);
  FC_LAUNCHED("k_select_dense64");
  return FC_OK;
}

}  // extern "C"

template <typename T>
static int mask_dense64(const T* g, uint64_t n, int codec, const uint32_t* mask_bits, double p,
                        uint64_t seed, uint64_t offset, double* out, fc_stream_t stream) {
  FC_CHECK(g && out, "NULL argument");
  FC_CHECK(n >= 1 && n <= 0xffffffffull, "n=%llu outside [1, 2^32-1]", (unsigned long long)n);
  FC_CHECK(codec == FC_CODEC_DROPOUT_BIASED || codec == FC_CODEC_DROPOUT_UNBIASED ||
               codec == FC_CODEC_RAND, "bad codec %d", codec);
  FC_CHECK(mask_bits || codec != FC_CODEC_RAND, "native rand-k uses fc_topk_dense_f64(PHILOX)");
  FC_CHECK(mask_bits || (p >= 0.0 && p <= 1.0), "p=%g outside [0, 1]", p);
  double thr = floor(p * 4294967296.0 + 0.5);
  if (thr < 0) thr = 0;
  if (thr > 4294967296.0) thr = 4294967296.0;
  const int mode = codec == FC_CODEC_RAND ? 0 : codec == FC_CODEC_DROPOUT_BIASED ? 1 : 2;
  hipStream_t s = (hipStream_t)stream;
  TimedLaunch t(FC_TIME_COMPACT, s);
  hipLaunchKernelGGL(k_mask_dense64<T>, dim3(grid_of((n + 3) / 4)), dim3(kBlock), 0, s, g, n, mask_bits,
                     (uint64_t)thr, seed, offset, mode, p, out);
  FC_LAUNCHED("k_mask_dense64");
  return FC_OK;
}

extern "C" {

int fc_mask_dense_f64(const double* g, uint64_t n, int codec, const uint32_t* mask_bits, double p,
                      uint64_t seed, uint64_t offset, double* out, fc_stream_t stream) {
  return mask_dense64(g, n, codec, mask_bits, p, seed, offset, out, stream);
}

int fc_mask_dense_f32(const float* g, uint64_t n, int codec, const uint32_t* mask_bits, double p,
                      uint64_t seed, uint64_t offset, double* out, fc_stream_t stream) {
  return mask_dense64(g, n, codec, mask_bits, p, seed, offset, out, stream);
}

int fc_weighted_sum_dense_f64(const void* const* rows, int rows_f64, const double* w, int m,
                              uint64_t n, double* out, int continue_sum, fc_stream_t stream) {
  FC_CHECK(rows && w && out, "NULL argument");
  FC_CHECK(m >= 1, "m=%d < 1", m);
  FC_CHECK(n >= 1, "n=0");
  hipLaunchKernelGGL(k_wsum64, dim3(grid_of(n)), dim3(kBlock), 0, (hipStream_t)stream, rows,
                     rows_f64, w, m, n, out, continue_sum);
  FC_LAUNCHED("k_wsum64");
  return FC_OK;
}

int fc_div_scalar_f64(double* x, uint64_t n, double d, fc_stream_t stream) {
  FC_CHECK(x != nullptr, "x is NULL");
  FC_CHECK(n >= 1, "n=0");
  hipLaunchKernelGGL(k_div_scalar64, dim3(grid_of(n)), dim3(kBlock), 0, (hipStream_t)stream, x, n, d);
  FC_LAUNCHED("k_div_scalar64");
  return FC_OK;
}

}  // extern "C"
