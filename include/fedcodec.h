/* fedcodec.h — C ABI of the MI355X-native gradient codec (libfedcodec.so, gfx950).
 *
 * Replaces the NumPy kernels inside OpenMSFTL's ftl/compression + FedAVG hot path:
 *   Compression.compress          ftl/compression/compression.py:23-77
 *     'top'              -> fc_topk_encode (+ fc_topk_encode_exact)   compression.py:31-37
 *     'rand'             -> fc_topk_encode (key_mode = PHILOX, native) or
 *                           fc_mask_encode (host permutation mask, parity)  compression.py:39-45
 *     'dropout-biased'   -> fc_mask_encode (codec = DROPOUT_BIASED)   compression.py:47-53
 *     'dropout-unbiased' -> fc_mask_encode (codec = DROPOUT_UNBIASED) compression.py:55-60
 *     dense result       -> fc_decode_dense
 *   Aggregator.aggregate_grads G build   aggregation.py:61-63   -> fc_decode_accumulate
 *   GAR.weighted_average / FedAvg        gar.py:32-46, 53-56    -> fc_decode_accumulate /
 *                                                                  fc_weighted_sum_dense
 *   flatten_params / client delta        model_helper.py:11-35,
 *                                        client.py:44,52-53     -> fc_flat_stage
 *   Aggregator.__merge_gradient          aggregation.py:80-93   -> fc_decode_accumulate /
 *                                                                  fc_weighted_sum_dense (w=1)
 *                                                                  + fc_div_scalar
 * The reference has no FFI of its own (100 % Python): these entry points are
 * what its Python layer binds through ctypes.
 *
 * Conventions: every pointer is a DEVICE pointer unless stated; buffers are caller-owned;
 * calls are stream-ordered and asynchronous; nothing allocates (scratch lives in the caller's
 * workspace); return 0 on success, <0 on argument / HIP errors (fc_last_error() explains,
 * thread-local).  Device-side outcomes (e.g. the sampled bracket missing) are reported in the
 * packet header's `status`, read by the host after the stream is synchronised.
 *
 * Concurrency: every entry point may run beside any other kernel, on any stream.  Two
 * launches wait in-kernel (bounded) for a bracket their own sample workgroups publish: k_fused_mag
 * (fc_topk_encode with key_mode MAGNITUDE and 0 < k < n, fc_topk_encode_dense) and k_fused64
 * (fc_topk_dense_f64_sampled).  Two of them on two streams of one device could stall each other
 * (each XCD dispatches the two grids in its own order), so the library queues each one after the
 * device's previous one: an event it owns completes with every such launch, and a launch on
 * another stream first waits for it.  A launch into a stream being captured (hipGraph) is not
 * ordered; bracket the graph's launch with fc_fused_order_begin / fc_fused_order_end.  All other
 * kernels synchronise only through last-arriver tickets (no workgroup waits for another).
 */
#ifndef FEDCODEC_H_
#define FEDCODEC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* fc_stream_t; /* hipStream_t */

/* ABI history: 2 = per-chunk quarter offsets (qoff); 3 = uint16 chunk-local packet indices;
 * 4 = fc_topk_encode_dense's packet is scratch (no entries; header format FC_FMT_DENSE, which
 * the decode entry points must not be given: they trust the caller's format argument).  A C
 * caller built against 3 that decoded that packet must check this version. */
#define FC_ABI_VERSION 4

/* return codes */
#define FC_OK 0
#define FC_ERR_ARG (-1)
#define FC_ERR_HIP (-2)
#define FC_ERR_WORKSPACE (-3)

/* packet header status (device-written) */
#define FC_STATUS_OK 0
#define FC_STATUS_RETRY_EXACT 1   /* sampled bracket missed: call fc_topk_encode_exact */
#define FC_STATUS_OVERFLOW 2      /* more entries than the packet capacity */
#define FC_STATUS_TIMEOUT 3       /* a bounded device spin expired (never expected) */

/* codecs (compression_function) */
#define FC_CODEC_TOP 1
#define FC_CODEC_RAND 2
#define FC_CODEC_DROPOUT_BIASED 3
#define FC_CODEC_DROPOUT_UNBIASED 4
#define FC_CODEC_QSGD 5      /* opt-in: the reference raises NotImplementedError (:62-64)    */

/* key sources for fc_topk_encode */
#define FC_KEY_MAGNITUDE 0   /* |g| (top-k) */
#define FC_KEY_PHILOX 1      /* Philox4x32-10 word per element (native rand-k) */

/* packet formats */
#define FC_FMT_IDXVAL 0      /* uint16 idx[] (chunk-local, ascending) + float val[] */
#define FC_FMT_BITMAP 1      /* uint32 bitmap[ceil(N/8192)*256] + float val[] */
#define FC_FMT_QSGD 2        /* packed W-bit codes (sign | level), fc_qsgd_code_words */
#define FC_FMT_DENSE 3       /* header of fc_topk_encode_dense: the dense q is the product;
                                idx/val/cnt/qoff are scratch (not a decodable packet) */

/* Slotted packet layout: the gradient is cut into chunks of FC_CHUNK elements; chunk c's
 * entries (ascending index order) live at [c*FC_CHUNK, c*FC_CHUNK + cnt[c]) of idx/val (and
 * its bitmap words at [c*256, c*256+256)).  idx holds the CHUNK-LOCAL index (uint16, the
 * element is c*FC_CHUNK + idx): 6 bytes per entry instead of 8 (ABI 3).  Every chunk is encoded by an independent
 * workgroup — no global scan — so buffers are sized fc_packet_capacity(n) entries while only
 * the listed entries are written or read.
 * FC_FMT_IDXVAL packets also carry qoff[c] (uint64 per chunk): the slot positions where the
 * chunk's four quarters (FC_CHUNK/4 elements each) begin — quarter 1, 2, 3 in bits 0-15,
 * 16-31, 32-47 — and cnt[c] in bits 48-63, so a decoder can hand each quarter to its own wave
 * (fc_decode_accumulate requires it). */
#define FC_CHUNK 8192        /* elements per chunk */
#define FC_QUARTER (FC_CHUNK / 4)

/* Device-resident packet header (96 bytes). */
typedef struct fc_packet_hdr {
  uint64_t thresh;      /* T64: entry kept iff (key<<index_bits | index) >= thresh    */
  uint64_t lower;       /* L64: every element with comp >= lower is listed             */
  uint32_t n;           /* gradient length                                             */
  uint32_t k;           /* coordinates kept by the codec (top/rand)                    */
  uint32_t n_entries;   /* entries listed (sum of cnt; >= k: sampled-bracket slack)    */
  uint32_t index_bits;  /* IB = max(1, ceil(log2 n))                                   */
  uint32_t codec;       /* FC_CODEC_*                                                  */
  uint32_t status;      /* FC_STATUS_*                                                 */
  uint32_t n_definite;  /* diagnostics: elements above the bracket                     */
  uint32_t n_cand;      /* diagnostics: elements inside the bracket                    */
  uint64_t seed;        /* Philox key (native RNG modes)                               */
  uint64_t offset;      /* Philox counter high words                                   */
  double p;             /* dropout probability (unbiased scale 1/p applied at decode)  */
  uint32_t chunk;       /* FC_CHUNK                                                    */
  uint32_t format;      /* FC_FMT_*                                                    */
  uint32_t key_mode;    /* FC_KEY_* (top/rand)                                         */
  uint32_t reserved[3];
} fc_packet_hdr;

/* One packet as seen by the decoders (host- or device-resident array element, 56 bytes). */
typedef struct fc_packet_view {
  const void* idx;              /* FC_FMT_IDXVAL: uint16 chunk-local indices; FC_FMT_QSGD: uint32 codes */
  const float* val;
  const uint32_t* bitmap;       /* FC_FMT_BITMAP                        */
  const uint32_t* cnt;          /* ceil(N/FC_CHUNK) entries per chunk   */
  const fc_packet_hdr* hdr;
  const uint64_t* qoff;         /* FC_FMT_IDXVAL: quarter offsets per chunk (see above) */
  float weight;                 /* FedAVG weight w_i (gar.py:37-44)     */
  uint32_t reserved;
} fc_packet_view;

int fc_abi_version(void);
const char* fc_last_error(void);

/* ---- sizes ------------------------------------------------------------------------- */
uint64_t fc_num_chunks(uint64_t n);
size_t fc_workspace_bytes(uint64_t n);        /* scratch for one encoder (one stream)   */
uint64_t fc_packet_capacity(uint64_t n);      /* idx/val entries: ceil(n/FC_CHUNK)*FC_CHUNK */
/* zero a freshly allocated workspace once (self-cleaning afterwards) */
int fc_workspace_init(void* ws, size_t ws_bytes, fc_stream_t stream);

/* ---- encode: top-k / native rand-k (compression.py:31-45) ---------------------------
 * Single streaming read of g: a sampled bracket [t_lo, t_hi] is estimated from a
 * stratified sample, every element with key >= t_lo is compacted in index order into its
 * chunk's slot (one launch, independent workgroups), then the exact k-th composite key is
 * resolved from the bracket's candidates.  hdr->status == FC_STATUS_RETRY_EXACT means the
 * bracket missed (adversarial / tie-heavy data): call fc_topk_encode_exact with the same
 * arguments.  capacity >= fc_packet_capacity(n); cnt and qoff have fc_num_chunks(n) words
 * (qoff may be NULL: not written; fc_decode_accumulate then folds the packet by scanning each
 * chunk's whole slot range per quarter, correct but slower). */
int fc_topk_encode(const float* g, uint64_t n, uint64_t k, int key_mode, uint64_t seed,
                   uint64_t offset, uint16_t* idx, float* val, uint64_t capacity,
                   uint32_t* cnt, uint64_t* qoff, fc_packet_hdr* hdr, void* ws, size_t ws_bytes,
                   fc_stream_t stream);
/* ---- top-k straight to the dense result (compression.py:31-37 returns q, not a packet) --
 * The fc_topk_encode pipeline (magnitude keys) whose compaction pass also streams
 * q = zeros_like(g); q[listed] = g into `dense` (n floats, 16-B aligned); the resolve zeroes
 * the slack entries once T64 is known.  q is the product: the packet buffers are scratch (the
 * entries are written only for chunks the resolve has to re-read) and the header's format is
 * FC_FMT_DENSE (thresh / status valid; not decodable).  If the header reports
 * FC_STATUS_RETRY_EXACT, `dense` is not valid: re-encode with fc_topk_encode_exact (a full
 * packet) and fc_decode_dense.  Needs 0 < k < n. */
/* fc_topk_encode_decode: the packet encode of fc_topk_encode (key_mode MAGNITUDE, 0 < k < n,
 * qoff required) AND its dense decode into out (float32[n], 16-B aligned), with the resolve's
 * gather and finish inside the decode launch (k_fused_mag -> k_beta -> k_decode_res): the packet
 * (entries, counts, quarter offsets, header with T64) equals fc_topk_encode's byte for byte and
 * out equals fc_decode_dense of it.  Replaces compression.py:31-37 + the caller's use of q.
 * Header status FC_STATUS_RETRY_EXACT: call fc_topk_encode_exact, then fc_decode_dense. */
int fc_topk_encode_decode(const float* g, uint64_t n, uint64_t k, uint16_t* idx, float* val,
                          uint64_t capacity, uint32_t* cnt, uint64_t* qoff, fc_packet_hdr* hdr,
                          void* ws, size_t ws_bytes, float* out, fc_stream_t stream);
int fc_topk_encode_dense(const float* g, uint64_t n, uint64_t k, uint16_t* idx, float* val,
                         uint64_t capacity, uint32_t* cnt, uint64_t* qoff, fc_packet_hdr* hdr,
                         void* ws, size_t ws_bytes, float* dense, fc_stream_t stream);
/* ---- batched top-k / native rand-k: M clients, one launch per pipeline stage ----------
 * The same fast path as fc_topk_encode for m gradients of equal length n, with the grid's
 * y dimension indexing the client: 4 launches for the whole batch instead of 4 per client,
 * so the small sampling / resolve stages of all clients overlap.  jobs: DEVICE array of m
 * fc_encode_job; ws: fc_workspace_bytes_batch(n, m) bytes, zeroed once with
 * fc_workspace_init.  Requires 0 < k < n (trivial k: fc_topk_encode).  A packet whose header
 * reports FC_STATUS_RETRY_EXACT is re-encoded with fc_topk_encode_exact, as for one client. */
typedef struct fc_encode_job {
  const float* g;        /* gradient, 16-B aligned                          */
  uint16_t* idx;         /* packet buffers (capacity >= fc_packet_capacity) */
  float* val;
  uint32_t* cnt;
  fc_packet_hdr* hdr;
  uint64_t seed;         /* Philox key / counter (FC_KEY_PHILOX)            */
  uint64_t offset;
  uint64_t* qoff;        /* quarter offsets per chunk (may be NULL)         */
} fc_encode_job;         /* 64 bytes */
size_t fc_workspace_bytes_batch(uint64_t n, int m);
int fc_topk_encode_batch(const fc_encode_job* jobs_dev, int m, uint64_t n, uint64_t k,
                         int key_mode, uint64_t capacity, void* ws, size_t ws_bytes,
                         fc_stream_t stream);
/* The same pipeline in two parts on the caller's stream (the same jobs and ws for both):
 * FC_PART_SAMPLE launches the bracket sample, which reads g and writes only the headers and
 * the workspace; FC_PART_FINISH launches the compaction and the exact resolve, which write the
 * packet buffers.  A caller that double-buffers the headers can therefore run the next
 * batch's sample while the previous packets are still being read (fc_decode_accumulate), and
 * order FC_PART_FINISH behind that fold.  part = FC_PART_SAMPLE | FC_PART_FINISH is
 * fc_topk_encode_batch. */
#define FC_PART_SAMPLE 1
#define FC_PART_FINISH 2
int fc_topk_encode_batch_part(const fc_encode_job* jobs_dev, int m, uint64_t n, uint64_t k,
                              int key_mode, uint64_t capacity, void* ws, size_t ws_bytes,
                              int part, fc_stream_t stream);

/* Exact radix-select path (several reads of g); always succeeds; n_entries == k. */
int fc_topk_encode_exact(const float* g, uint64_t n, uint64_t k, int key_mode, uint64_t seed,
                         uint64_t offset, uint16_t* idx, float* val, uint64_t capacity,
                         uint32_t* cnt, uint64_t* qoff, fc_packet_hdr* hdr, void* ws,
                         size_t ws_bytes, fc_stream_t stream);

/* ---- encode: mask codecs (compression.py:39-60) -------------------------------------
 * codec = FC_CODEC_DROPOUT_* or FC_CODEC_RAND (parity mode: mask from the host's
 * np.random.permutation).  mask_bits (little-endian bit i = element i, N/32 words) is the
 * host-drawn mask in parity mode; NULL selects native Philox Bernoulli(p) keyed by seed.
 * format: FC_FMT_BITMAP (bitmap required) or FC_FMT_IDXVAL (idx required; qoff written when
 * non-NULL). */
int fc_mask_encode(const float* g, uint64_t n, int codec, const uint32_t* mask_bits,
                   double p, uint64_t seed, uint64_t offset, int format, uint16_t* idx,
                   float* val, uint32_t* bitmap, uint64_t capacity, uint32_t* cnt,
                   uint64_t* qoff, fc_packet_hdr* hdr, void* ws, size_t ws_bytes,
                   fc_stream_t stream);

/* ---- decode (compression.py dense result) --------------------------------------------
 * pkt: HOST pointer to one view.  out is float (out_f64 = 0) or double (out_f64 = 1; the
 * reference's float64 dropout result, compression.py:52/60). */
int fc_decode_dense(const fc_packet_view* pkt, int format, uint64_t n, void* out, int out_f64,
                    fc_stream_t stream);

/* ---- FedAVG over packets (aggregation.py:61-63 + gar.py:44), bit-exact fp32 ----------
 * views: DEVICE array of m views (same format), client order = row order of G; FC_FMT_IDXVAL
 * each chunk quarter is folded by its own wave with no barrier, using the views' qoff (a view
 * without qoff is folded by whole-chunk scans).
 * acc[j] = fl(w_0 * d_0[j]);  acc[j] = fl(acc[j] + fl(w_i * d_i[j])) for i = 1..m-1. */
int fc_decode_accumulate(const fc_packet_view* views_dev, int m, int format, uint64_t n,
                         float* acc, fc_stream_t stream);
/* Same fold, continuing the partial sum already held in acc (acc = fl(acc + fl(w_i * d_i))
 * for i = 0..m-1): rows of G split across calls or across GPUs (the exact chained reduce of
 * SURVEY.md §8(e)) give the same bits as one call over all rows. */
int fc_decode_accumulate_continue(const fc_packet_view* views_dev, int m, int format,
                                  uint64_t n, float* acc, fc_stream_t stream);

/* ---- FedAVG over dense rows (gar.py:44 for 'full'): rows = DEVICE array of m row
 * pointers, w = DEVICE fp32[m]. */
int fc_weighted_sum_dense(const float* const* rows, const float* w, int m, uint64_t n,
                          float* out, fc_stream_t stream);
/* Same sum continuing the partial sum already in out (out = fl(out + fl(w_i * row_i)) for
 * i = 0..m-1): 'full' rows streamed group by group from host memory (aggregation.py:61-63)
 * fold to the same bits as one call over all rows. */
int fc_weighted_sum_dense_continue(const float* const* rows, const float* w, int m, uint64_t n,
                                   float* out, fc_stream_t stream);

/* ---- flat-layout staging on the device (model_helper.py:11-35, client.py:44,52-53) ------
 * params_dev: DEVICE array of `count` fp32 parameter pointers; offsets_dev: DEVICE
 * uint64[count + 1] prefix offsets into the flat vector (max_size = largest parameter).
 * scatter = 0: flat[off_p + i] <- param_p[i]; with grad != NULL first
 *   grad = fl32(flat_old - param)  (client.py:53: current_weights - updated_model_weights),
 *   i.e. flatten_params + the client delta in one pass, flat keeping the new weights;
 * scatter = 1: param_p[i] <- flat[off_p + i]  (dist_weights_to_model / dist_grads_to_model). */
int fc_flat_stage(const float* const* params_dev, const uint64_t* offsets_dev, int count,
                  uint64_t max_size, float* flat, float* grad, int scatter, fc_stream_t stream);

/* ---- hierarchical merge (aggregation.py:80-93): a cluster's mean
 * np.mean(G[s:e, :], axis=0) is the +0-started row-order sum (fc_decode_accumulate /
 * fc_weighted_sum_dense with weights 1.0) divided once by the row count: x = fl(x / d), in
 * place, x a DEVICE fp32[n] (16-B aligned). */
int fc_div_scalar(float* x, uint64_t n, float d, fc_stream_t stream);

/* ---- QSGD quantiser (compression.py:62-74, the reference's commented formula; opt-in,
 * parity unpinned with respect to the reference, pinned to oracle/qsgd_oracle.py) ------
 * q_i = sign(g_i) * ||g|| / (s tau) * floor(s |g_i| / ||g|| + U_i), s = 2^bits (1..14),
 * tau = 1 + min(sqrt(n)/s, n/s^2), U_i from Philox(seed, offset).  Codes: W = 4/8/16-bit
 * (sign | level) packed little-endian into code_words >= fc_qsgd_code_words(n, bits) uint32
 * (16-B aligned).  The header records ||g|| (double, field p), bits (field k), the Philox
 * key/counter, codec FC_CODEC_QSGD and format FC_FMT_QSGD.  ws: fc_qsgd_workspace_bytes(),
 * zeroed once.  Decoders take fc_packet_view with idx = codes. */
uint64_t fc_qsgd_code_words(uint64_t n, int bits);
size_t fc_qsgd_workspace_bytes(void);
int fc_qsgd_encode(const float* g, uint64_t n, int bits, uint64_t seed, uint64_t offset,
                   uint32_t* codes, uint64_t code_words, fc_packet_hdr* hdr, void* ws,
                   size_t ws_bytes, fc_stream_t stream);
int fc_qsgd_decode(const fc_packet_view* pkt, uint64_t n, float* out, fc_stream_t stream);
/* FedAVG over QSGD packets (views_dev: DEVICE array of m views, weights in the views):
 * out = fl(... fl(+0 + fl(w_0 q_0)) ...) in row order (gar.py:44); continue_sum != 0 folds
 * into the partial sum already in out. */
int fc_qsgd_decode_accumulate(const fc_packet_view* views_dev, int m, uint64_t n, float* out,
                              int continue_sum, fc_stream_t stream);

/* ---- float64 gradients ------------------------------------------------------------
 * The reference reaches the codec with float64 gradients after RandomGaussian with
 * noise_scale == 0 (attack_models.py:105-106); G takes that dtype (aggregation.py:61) and
 * every codec and gar.py:44 then compute in float64.  These entry points produce the dense
 * float64 result compress() returns (all buffers DEVICE, float64, 8-B aligned).
 * fc_topk_dense_f64: 'top' (key_mode MAGNITUDE) / native 'rand' (PHILOX), exact radix select
 *   of the k-th largest (key64 << 32 | idx) (<= 8 passes over g) then q = selected ? g : +0;
 *   same tie rule as the fp32 path.  ws: fc_workspace_bytes(n), zeroed once.
 * fc_mask_dense_f64: codec RAND (mask_bits required: q = keep ? g : +0), DROPOUT_BIASED
 *   (q = g * keep) or DROPOUT_UNBIASED (q = (g * keep) / p), the reference's float64
 *   arithmetic including -0 and NaN (inf * 0); mask_bits NULL = native Philox Bernoulli(p).
 * fc_mask_dense_f32: the same on a float32 gradient (4-B aligned), promoted exactly: the
 *   float64 array compression.py:47-60 returns for float32 client.grad, -0.0 included
 *   (replaces compression.py:51-53 / :58-60 on the drop-in path).
 * fc_weighted_sum_dense_f64: gar.py:44 when G or the weights are float64: rows = DEVICE
 *   array of m row pointers (float32 if rows_f64 == 0, promoted exactly), w = DEVICE
 *   float64[m]; out = +0-started row-order fp64 sum of fl64(g_i * w_i); continue_sum != 0
 *   continues the sum already in out.
 * fc_div_scalar_f64: x = fl64(x / d) in place (np.mean's count division for float64 G).
 * fc_topk_dense_f64_sampled: 'top' (magnitude keys, 0 < k < n, g / out 16-B aligned) by the
 *   fp32 design on each double's high 31-bit key: sampled bracket, ONE streaming pass that
 *   writes out and lists the bracket's candidates, exact select among them, slack fix-up
 *   (replaces compression.py:31-37 for float64 client.grad; 8N read + 8N written instead of
 *   <= 8 passes of 8N).  Writes *status (DEVICE uint32) = FC_STATUS_OK, or
 *   FC_STATUS_RETRY_EXACT when the bracket missed (or > 2048 candidates share the rank's
 *   histogram bin): out is then not valid and the caller runs fc_topk_dense_f64 (exact).  Same result bits as
 *   fc_topk_dense_f64.  ws: fc_workspace_bytes(n), zeroed once. */
int fc_topk_dense_f64_sampled(const double* g, uint64_t n, uint64_t k, double* out, void* ws,
                              size_t ws_bytes, uint32_t* status, fc_stream_t stream);
int fc_topk_dense_f64(const double* g, uint64_t n, uint64_t k, int key_mode, uint64_t seed,
                      uint64_t offset, double* out, void* ws, size_t ws_bytes,
                      fc_stream_t stream);
int fc_mask_dense_f64(const double* g, uint64_t n, int codec, const uint32_t* mask_bits, double p,
                      uint64_t seed, uint64_t offset, double* out, fc_stream_t stream);
int fc_mask_dense_f32(const float* g, uint64_t n, int codec, const uint32_t* mask_bits, double p,
                      uint64_t seed, uint64_t offset, double* out, fc_stream_t stream);
int fc_weighted_sum_dense_f64(const void* const* rows, int rows_f64, const double* w, int m,
                              uint64_t n, double* out, int continue_sum, fc_stream_t stream);
int fc_div_scalar_f64(double* x, uint64_t n, double d, fc_stream_t stream);

/* ---- NumPy's legacy MT19937 stream on the device: the reference's own dropout draws ---------
 * Replaces np.random.binomial(1, p, (n,)) of compression.py:51 / :58 (the process-global legacy
 * RandomState; NumPy's random_binomial_inversion for n = 1: U = random_sample() from two
 * 32-bit outputs, kept iff U > exp(log(1 - p)), complemented for p > 0.5).  A round draws the
 * masks of `rows` consecutive dropout rows of length n, row r starting 2 r n outputs after the
 * state (key, pos) of np.random.get_state(); the mask words equal
 * bitmask_words(np.random.binomial(1, p, (n,)), n, True) bit for bit, and the state block
 * holds the state np.random would be left in (openmsftl_amd/csrc/fc_mt.hip; pinned against
 * NumPy in tests/test_mt19937.py).
 *   fc_mt_plan: the jump polynomials of length n for up to `rows` rows (computed on the host,
 *     cached per n; the first n costs ~0.1-0.5 s) copied into the DEVICE buffer `plan`
 *     (fc_mt_plan_bytes); synchronises `stream`.  Reusable for every round of length n and
 *     at most `rows` rows.
 *   fc_mt_begin: the round's starting state (key: HOST uint32[624], pos in [0, 624]) into
 *     the DEVICE workspace (fc_mt_workspace_bytes(rows), 256-B aligned), each row's window
 *     and raw sequence, and the state after `rows` rows into the fc_mt_state at ws offset 0.
 *   fc_mt_binomial: row `row`'s mask (mask_bits: DEVICE uint32[ceil(n/32)], bits >= n zero),
 *     after fc_mt_begin on the same stream.  p outside [0, 1] is FC_ERR_ARG (NumPy raises
 *     ValueError).  NumPy's rare redraw (U - qn > p qn / (1 - p) after U > qn, ~2^-52 per
 *     element) is not reproduced: fc_mt_state.redraw becomes non-zero and the caller must draw
 *     the round on the host instead.
 *   fc_mt_jump_poly / fc_mt_charpoly (HOST, no GPU): z^d mod chi and chi (MT19937's
 *     characteristic polynomial, degree 19937) as 624 little-endian words (bit i = z^i). */
#define FC_MT_SEG 32768           /* mask elements per generator wave */
typedef struct {
  uint32_t key[624];              /* np.random.get_state()[1] after the round */
  uint32_t pos;                   /* ... [2] */
  uint32_t redraw;                /* != 0: NumPy would have redrawn: use host draws */
  uint32_t rows;
  uint32_t start_pos;
} fc_mt_state;
size_t fc_mt_plan_bytes(uint64_t n, int rows);
size_t fc_mt_workspace_bytes(int rows);
int fc_mt_plan(uint64_t n, int rows, void* plan, size_t plan_bytes, fc_stream_t stream);
int fc_mt_begin(const void* plan, size_t plan_bytes, uint64_t n, int rows, const uint32_t* key,
                uint32_t pos, void* ws, size_t ws_bytes, fc_stream_t stream);
int fc_mt_binomial(const void* plan, size_t plan_bytes, uint64_t n, int rows, int row, double p,
                   uint32_t* mask_bits, void* ws, size_t ws_bytes, fc_stream_t stream);
int fc_mt_jump_poly(uint64_t d, uint32_t* out_words);
int fc_mt_charpoly(uint32_t* out_words);

/* Ordering of in-kernel-waiting launches issued outside the library's own calls (a replayed
 * graph that contains fc_topk_encode / fc_topk_encode_dense / fc_topk_dense_f64_sampled):
 * fc_fused_order_begin(s) makes s wait for the device's last such launch; fc_fused_order_end(s)
 * marks s as holding the latest one. */
int fc_fused_order_begin(fc_stream_t stream);
int fc_fused_order_end(fc_stream_t stream);

/* ---- measurement: HIP events around selected kernels, on the stream they run on -------
 * mask: FC_TIME_* bits.  Between fc_timing_begin and fc_timing_end every launch of a
 * selected kernel class is bracketed by a hipEvent pair; fc_timing_end synchronises those
 * events and returns per-class total milliseconds and launch counts (arrays of 4). */
#define FC_TIME_COMPACT 1    /* k_compact: the single streaming pass over g (encode)   */
#define FC_TIME_DECODE 2     /* k_decode: dense decode / FedAVG decode-accumulate      */
#define FC_TIME_ENGINE 4     /* k_engine: exact threshold resolution                   */
#define FC_TIME_SAMPLE 8     /* k_sample: bracket estimation                           */
int fc_timing_begin(uint32_t mask);
int fc_timing_end(double* total_ms, uint64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* FEDCODEC_H_ */
