// fc_state.h — encoder workspace layout + shared argument blocks (device and host views).
#pragma once
#include <stdint.h>
#include "../../include/fedcodec.h"
#include "fc_common.h"

namespace fc {

// Per-encoder state.  Self-cleaning: every counter a kernel consumes is reset by the
// workgroup that consumed it last, so a stream of encodes (or a graph replay) needs the
// workspace zeroed only once (fc_workspace_init).
struct alignas(16) TopkState {
  uint64_t ticket;       // k_compact chunk tickets {epoch:32 | count:32}; the holder of the
                         // last ticket starts the next epoch at count 0
  uint64_t L64;          // entries written: comp >= L64
  uint64_t e_prefix;     // exact radix engine: resolved high bits of T64
  uint32_t err;          // sticky device error (spin timeout)
  uint32_t a_done, b_done, r_done;
  uint32_t pad0_[3];
  uint32_t win_flag;     // batched encode: k_pilot's fine window for k_sample1 (bit 31 valid,
                         // level-1 bins hi << 12 | lo; k_fused_mag's live in WsPtrs::pub)
  uint32_t pad1_[2];
  uint32_t t_lo, t_hi;   // bracket (keys): list key >= t_lo; candidates key <= t_hi
  uint32_t sbin;         // candidate histogram bin = (key - t_lo) >> sbin  (< 4096 bins)
  uint32_t cand_on, n_cand, cand_over, ent_over;
  uint32_t small_n;      // survivors gathered for the LDS finish
  uint32_t e_shift, e_rank, e_matched, e_done, e_ticket, e_status;
  uint32_t gen;          // k_resolve generation: bumped when T64 is published (dense fix-up)
  uint32_t small_done;   // k_decode_res: bin-beta entries stored (the last one finishes T64)
  uint32_t fz_seq;       // k_fused_mag launches completed (bumped by the following k_resolve);
                         // a launch tags its bracket records (fz_seq + 1) | bit 31
  uint32_t hgen;         // k_resolve: bumped once the bin beta below is published
  uint32_t rb_beta, rb_rin, rb_cnt;   // k_resolve: bin holding rank r, rank inside it, its count
  uint32_t rb_flags;     // k_beta: bit 0 retry (exact path), bit 1 rank 0 (every candidate slack)
  uint32_t rb_nent, rb_ncand;         // k_beta: entries listed, candidates among them
  uint32_t shard_ent[kShards];   // k_compact totals, 64-way sharded (no hot word)
  uint32_t shard_cnd[kShards];
};
static_assert(sizeof(TopkState) <= 1024, "state block");

// Histogram shards (the sample's and the resolve's candidate histogram): fewer shards queue more
// same-address flush atomics but give the last arriver fewer loads, and its loads are on the
// latency chain.  Measured (profiles/r04_ab_hist_shards.jsonl): lone 16 M dense encode 57.5 ->
// 52 us with ONE sample shard for its 128 sample workgroups, 128 M best at two; the batched
// resolve 84 -> 78 us and the lone packet resolve 24 -> 23 us with two candidate shards (one:
// 26 us); eight candidate shards +50 %.
constexpr int FC_SAMPLE_SHARDS = 2;
constexpr int FC_CAND_SHARDS = 2;
constexpr int kSampleShards = FC_SAMPLE_SHARDS;   // k_sample1's global histogram, sharded by workgroup
constexpr int kCandShards = FC_CAND_SHARDS;       // k_resolve's candidate histogram, likewise
constexpr int kTickGroups = 16;             // two-level last-arriver tickets (fc_common.h)
constexpr int kTickStride = 64;             // u32 per ticket counter (one 256-B line each)
constexpr int kTickWords = (kTickGroups + 1) * kTickStride;
// k_fused_mag's in-launch publications, each written to several 128-B lines that their pollers
// spread over (every poller on ONE line queued behind the others: ~900 chunk workgroups saw a
// 16 M encode's bracket over a 5 us spread, then each read the state in a second round trip):
//   bracket records: kPubCopies x {t_lo, t_hi, sbin, tag}, one 16-B store / load each
//   window flags:    kWinCopies x the pilot's window word (k_sample1's win_flag format)
constexpr int kPubCopies = 64;
constexpr int kWinCopies = 16;
constexpr int kPubStride = 32;              // u32 per copy (one 128-B line)
constexpr int kPubWords = (kPubCopies + kWinCopies) * kPubStride;

struct WsLayout {
  uint64_t nchunks, cand_cap;
  uint64_t off_hist1, off_tick, off_ehist, off_chist, off_small, off_smallv, off_pub, off_status,
      off_cand, bytes;
  __host__ __device__ static WsLayout of(uint64_t n) {
    WsLayout L;
    L.nchunks = (n + kChunk - 1) / kChunk;
    L.cand_cap = L.nchunks * kCandSlot;                // per-chunk candidate slots
    uint64_t o = 1024;
    L.off_hist1 = o;  o += 4ull * kHistBins * kSampleShards;
    L.off_tick = o;   o += 4ull * kTickWords * 3;      // sample, resolve (gather), resolve (bins)
    L.off_ehist = o;  o += 4ull * kHistBins;
    // 8 KB of padding before the candidate histogram, which the drop-in dense encode hits with
    // one device atomic per candidate while it streams: at offset 63,232 (no padding) the lone
    // 16 M dense encode took 55.6 us and 128 M 219 us, with 4 / 8 / 16 KB of padding 51 us and
    // 211-214 us (2 KB: no change) — an HBM channel / bank collision of those atomics with
    // another hot line of the launch (profiles/r04_ab_chist_offset.jsonl)
    o += 8192;
    L.off_chist = o;  o += 4ull * kHistBins * kCandShards;
    L.off_small = o;  o += 8ull * kSmallCap;
    L.off_smallv = o; o += 4ull * kSmallCap;        // k_decode_res: the gathered entries' values
    L.off_pub = o;    o += 4ull * kPubWords;        // n-independent, like every counter above
    L.off_status = o; o += 4ull * (L.nchunks ? L.nchunks : 1);   // per-chunk candidate counts
    o = (o + 15) & ~15ull;
    L.off_cand = o;   o += 8ull * L.cand_cap;
    L.bytes = (o + 255) & ~255ull;
    return L;
  }
};

struct HdrInit {          // static header fields, written by the first kernel of a pipeline
  uint64_t seed, offset;
  double p;
  uint32_t n, k, ib, codec, format, key_mode;
};

struct WsPtrs {
  TopkState* st;
  uint32_t *hist1, *tick, *ehist, *chist;   // hist1: kSampleShards x 4096; tick: 3 tickets
  uint64_t* small;
  uint32_t* smallv;        // k_decode_res: value bits of small[i]
  uint32_t* pub;           // k_fused_mag publications (kPubWords)
  uint32_t* ccnt;          // candidates per chunk (may exceed kCandSlot: overflowed chunk)
  uint64_t* cand;          // chunk c's candidates at [c * kCandSlot, + min(ccnt, kCandSlot))
  uint64_t cand_cap;
};

// Batched encode: client j's workspace starts j * ws_stride bytes after client 0's.
__device__ __forceinline__ WsPtrs ws_shift(WsPtrs W, uint64_t bytes) {
  W.st = reinterpret_cast<TopkState*>(reinterpret_cast<char*>(W.st) + bytes);
  W.hist1 = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(W.hist1) + bytes);
  W.tick = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(W.tick) + bytes);
  W.ehist = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(W.ehist) + bytes);
  W.chist = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(W.chist) + bytes);
  W.small = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(W.small) + bytes);
  W.smallv = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(W.smallv) + bytes);
  W.pub = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(W.pub) + bytes);
  W.ccnt = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(W.ccnt) + bytes);
  W.cand = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(W.cand) + bytes);
  return W;
}

__device__ __forceinline__ void write_hdr_static(fc_packet_hdr* h, const HdrInit& hi) {
  h->thresh = 0; h->lower = 0;
  h->n = hi.n; h->k = hi.k; h->n_entries = 0; h->index_bits = hi.ib;
  h->codec = hi.codec; h->status = FC_STATUS_OK; h->n_definite = 0; h->n_cand = 0;
  h->seed = hi.seed; h->offset = hi.offset; h->p = hi.p;
  h->chunk = kChunk; h->format = hi.format; h->key_mode = hi.key_mode;
  h->reserved[0] = h->reserved[1] = h->reserved[2] = 0;
}

// Sampling plan (host-computed, passed by value).
struct SamplePlan {
  uint64_t n;
  uint32_t nseg;       // 1024-element segments
  uint32_t full;       // 1: segments tile [0, n) exactly (n <= kFullSampleMax)
  int64_t r_hi, r_lo;  // 1-based ranks from the top inside the sample
  uint32_t hi_none, lo_all;
  uint32_t np;         // pilot segments (<= kPilotSegs): workgroup 0's own segments
  uint32_t pstride;    // their spacing = the sample grid (segment j*pstride, j < np)
  int64_t pr_hi, pr_lo;  // pilot ranks (1-based from the top) that bound the fine window
  uint32_t cbins_log2;   // candidate histogram bins used: the bracket's span >> sbin < 2^cbins_log2
  uint32_t segs;         // sample segments per workgroup group (<= kSampleSegs): 2 up to 32 M
                         // elements (more, shorter sample workgroups: a shorter bracket chain),
                         // 4 above (fewer flushes; profiles/r05_ab_sample_segs.jsonl)
};
constexpr int FC_SAMPLE_SEGS_PER_WG = 4;
constexpr int kPilotSegs = FC_SAMPLE_SEGS_PER_WG;   // >= P.segs: the pilot IS workgroup 0's share
constexpr uint64_t kFullSampleMax = 1ull << 20;

__host__ __device__ __forceinline__ uint64_t seg_start(const SamplePlan& P, uint32_t s) {
  if (P.full || P.nseg == 1) return (uint64_t)s * 1024;
  return ((uint64_t)s * (P.n - 1024) / (P.nseg - 1)) & ~3ull;
}
// pilot segment j (< P.np): workgroup 0's segment j (spread over the gradient: the sample's
// segments are stratified and workgroup 0 takes every pstride-th one)
__host__ __device__ __forceinline__ uint32_t pilot_seg(const SamplePlan& P, uint32_t j) {
  return j * P.pstride;
}

}  // namespace fc
