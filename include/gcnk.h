/*
 * gcnk.h — C-ABI of libgcnk.so, the MI355X (gfx950) kernels behind the
 * drop-in GraphConvolution / GCN modules.
 *
 * The reference (anargh-t/Graph-Convolutional-Networks-for-Text-Classification)
 * has no native code: every arithmetic site on its hot path is a call into
 * ATen.  Each entry point below replaces one of those call sites:
 *
 *   layer.py:102  support = th.spmm(infeatn, W)   sparse X  -> gcnk_spmm_csr_f32 (X in CSR)
 *                                                 dense  H  -> gcnk_gemm_f32 (fp32 MFMA)
 *   layer.py:106  output  = th.spmm(adj, support)          -> gcnk_spmm_csr_f32 (A-hat in CSR)
 *   layer.py:110  output + bias                             -> fused epilogue (GCNK_EPI_BIAS*)
 *   layer.py:182  th.relu                                   -> fused epilogue (GCNK_EPI_BIAS_RELU)
 *   layer.py:185  th.dropout(x, p, train)                   -> fused epilogue (GCNK_EPI_*_DROP*)
 *   autograd of :102/:106/:110 (trainer.py:361 loss.backward())
 *                  A^T g, X^T g                             -> gcnk_spmm_csr_f32 on cached transposes
 *                  H^T g, g W^T, relu/dropout mask          -> gcnk_gemm_f32 (+GCNK_GEMM_EPI_MASK_POS)
 *                  sum over rows of g  (bias grad)          -> gcnk_colsum_f32
 *   utils.py:196-203 / trainer.py:226-238 (COO tensors handed to th.spmm)
 *                                                           -> gcnk_coo_to_csr + gcnk_spmm_plan_build (one-time)
 *   utils.py:185-213 preprocess_adj / normalize_adj          -> gcnk_sym_normalize (device, bit-exact)
 *   utils.py:25-109  accuracy / macro_f1 counts              -> gcnk_class_stats (one launch, no per-class syncs)
 *   trainer.py:98-148 edge list -> symmetric adjacency        -> gcnk_edgelist_size / _csr (host, no networkx)
 *   layer.py:185 th.dropout keep-mask draw (CPU generator)    -> gcnk_bernoulli_mt19937 (host, same stream)
 *
 * Conventions
 *   - All pointers are DEVICE pointers unless a parameter says "host".
 *   - Dense matrices are row-major fp32 with an explicit leading dimension.
 *   - CSR uses int32 row pointers / column indices (callers check < 2^31);
 *     element offsets into dense matrices are 64-bit.
 *   - Every call is asynchronous on `stream` (a hipStream_t; NULL = default
 *     stream).  No entry point allocates or frees device memory, and none
 *     synchronises, except gcnk_spmm_plan_query which is documented as a
 *     one-time setup sync.  All entry points are safe to capture in a hipGraph.
 *   - Return 0 on success; GCNK_EARG (-1) bad argument/shape, GCNK_EUNSUP (-2)
 *     unsupported configuration, GCNK_EHIP (-3) HIP launch/runtime error.
 *     The message is in a thread-local buffer returned by gcnk_last_error().
 *   - Reentrant and thread-safe: no global mutable state besides the
 *     thread-local error text (and a per-kernel one-time LDS-limit attribute).
 *     Calls that may run concurrently (two streams, the autograd thread beside
 *     the caller's) must not share a workspace or a counter region; plans
 *     are read-only after gcnk_spmm_plan_build and may be shared freely.
 */
#ifndef GCNK_H_
#define GCNK_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GCNK_ABI_VERSION 12

#define GCNK_OK 0
#define GCNK_EARG (-1)
#define GCNK_EUNSUP (-2)
#define GCNK_EHIP (-3)

/* SpMM epilogues (applied once per finished output row element).
 * keep-mask semantics follow ATen's dropout (noise = bernoulli(1-p)/(1-p),
 * out = x * noise): an element is kept where mask != 0 and multiplied by
 * drop_scale. */
#define GCNK_EPI_NONE 0
#define GCNK_EPI_BIAS 1            /* + bias[col]                      layer.py:110 */
#define GCNK_EPI_BIAS_RELU 2       /* relu(. + bias)                   layer.py:110,182 */
#define GCNK_EPI_BIAS_RELU_DROP 3  /* relu(.+bias) * (mask?scale:0)    layer.py:110,182,185 */
#define GCNK_EPI_BIAS_RELU_HASH 4  /* as 3 with an in-kernel counter-based RNG mask */
/* HASH: element (r, c) is kept iff hash(seed, base + offset + r*ldm + c) <
 * keep_prob, base = *rng_base (a device uint64 read by the kernel; 0 when
 * rng_base is NULL).  A caller replaying a captured graph advances *rng_base
 * on the device after each call (the GCN module adds rows*ldm), so every
 * replay draws a fresh mask with no host involvement. */

/* GEMM epilogues */
#define GCNK_GEMM_EPI_NONE 0
#define GCNK_GEMM_EPI_BIAS 1
#define GCNK_GEMM_EPI_BIAS_RELU 2
#define GCNK_GEMM_EPI_MASK_POS 5   /* C = (R[m,n] > 0) ? acc*scale : 0   (relu+dropout backward) */

int gcnk_abi_version(void);
const char* gcnk_last_error(void);

/* ---------------------------------------------------------------------------
 * CSR SpMM:  C[M x F] = epi( A[M x K] (CSR) * B[K x F] )
 * Replaces th.spmm(adj, support) (layer.py:106) and th.spmm(X, W)
 * (layer.py:102, sparse X) and their autograd (A^T g, X^T g).
 *
 * The operand is converted once (gcnk_spmm_plan_build) into a ROW-UNIT + TILE
 * plan (magic 'GNK5'):
 *  - dense blocks: rows are grouped by off-diagonal degree class (factor-8
 *    buckets, row order within a class) into blocks of 64; a block whose
 *    nonzeros fill >= dense_threshold of its condensed column set (and use
 *    each such column twice on average) is stored densely over those
 *    columns (MFMA fragment order, chunks of 64 columns) and runs on fp32
 *    MFMA, each B row of a chunk staged once per block instead of gathered
 *    per nonzero; its rows' diagonal entries are kept aside and added in the
 *    epilogue; multi-chunk blocks are summed from partial slabs in order.
 *    dense_threshold > 1 disables the part (default callers pass 0.25).
 *
 *  - row units: the other rows.  A row of at most `ipc` nonzeros is one unit
 *    owned by one lane group (LPR lanes, each a 16-B column vector); a
 *    heavier row is cut into segments of about ipc * groups nonzeros (at most
 *    64), each owned by `groups` lane groups (the 64/LPR groups of a
 *    wavefront, or the 4 wavefronts of a workgroup when LPR = 64) that take
 *    interleaved nonzeros and meet in a fixed-order reduction; a row of
 *    several segments leaves one partial per segment and the last segment to
 *    finish (arrival counters in the caller's COUNTER REGION: int32
 *    gcnk_spmm_counter_bytes(header) bytes, zero on entry and left zero on
 *    return) sums them in segment order.
 * All sums have a fixed order (no float atomics): bitwise reproducible.
 * gcnk_spmm_groups(F, lanes_hint) gives the `groups` the kernels use for a
 * width F; a plan serves every F with that count.  The plan copies the
 * values: rebuild it when they change.  Building copies the CSR to the host
 * and synchronises `stream` (one-time setup).  The _host variants build the
 * same plan image from HOST arrays into host memory (no device needed).
 *
 * Plan header (16 int32, first words of the plan; gcnk_spmm_plan_query):
 *   0 magic 'GNK5'  1 M  2 K  3 groups  4 ipc  5 row units
 *   6 heavy segments  7 heavy rows of > 1 segment  8 tile chunks
 *   9 multi-chunk blocks  10 slabs  11 tile blocks  12 diagonal kept aside
 *   (0/1)  13 nnz  14 partial slots  15 chunk items of single-chunk tile blocks
 * (Rounds 2-3 also built a hub-split plan and a split-K plan for R8's doc-topic
 * operands; both measured slower than this plan and were removed in ABI 8 --
 * DESIGN.md keeps their numbers.)
 * ------------------------------------------------------------------------- */
int32_t gcnk_spmm_groups(int32_t F, int32_t lanes_hint);
int32_t gcnk_spmm_default_ipc(int32_t M, int64_t nnz, int32_t F, int32_t lanes_hint);
/* Size of the plan buffer (synchronises `stream`; negative error code on failure). */
int64_t gcnk_spmm_plan_bytes(const int32_t* rowptr, const int32_t* colind, int32_t M, int32_t K,
                             int64_t nnz, int32_t ipc, int32_t groups, float dense_threshold, void* stream);
int gcnk_spmm_plan_build(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t M,
                         int32_t K, int64_t nnz, int32_t ipc, int32_t groups, float dense_threshold,
                         void* plan, int64_t plan_bytes, void* stream);
/* The same from HOST arrays into a HOST buffer (plan-layout checks without a GPU). */
int64_t gcnk_spmm_plan_bytes_host(const int32_t* rowptr, const int32_t* colind, int32_t M, int32_t K,
                                  int64_t nnz, int32_t ipc, int32_t groups, float dense_threshold);
int gcnk_spmm_plan_build_host(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t M,
                              int32_t K, int64_t nnz, int32_t ipc, int32_t groups, float dense_threshold,
                              int32_t* plan, int64_t plan_bytes);
/* Copies the 16-word plan header to host memory `out16` and synchronises
 * `stream` (one-time setup).  Every SpMM call takes this host header. */
int gcnk_spmm_plan_query(const void* plan, int32_t* out16, void* stream);
/* Bytes of workspace (split-row partials, tile slabs) an SpMM of width F needs. */
int64_t gcnk_spmm_workspace_bytes(const int32_t* plan_header, int32_t F);
/* Bytes of the counter region a call needs (0: none).  The region is zeroed
 * ONCE by the caller and then used by calls on one stream in order (never
 * concurrently by two calls): the kernels leave it zero for the next call. */
int64_t gcnk_spmm_counter_bytes(const int32_t* plan_header);

/* C = epi(A B) for the operand of `plan` (M x K from the header). */
int gcnk_spmm_csr_f32(const void* plan, const int32_t* plan_header,
                      const float* B, int64_t ldb, int32_t F,
                      float* C, int64_t ldc,
                      const float* bias, int32_t epilogue,
                      const uint8_t* drop_mask, int64_t ldm, float drop_scale,
                      float keep_prob, uint64_t seed, uint64_t offset, const uint64_t* rng_base,
                      float* workspace, int64_t workspace_bytes,
                      int32_t* counters, int64_t counter_bytes,
                      int32_t lanes_hint, void* stream);

/* The same product in two parts that write disjoint rows of C, for callers
 * that overlap them on two streams (join both before reading C):
 *   part 1: the single-chunk dense tile blocks (plan header word 15 items);
 *   part 2: everything else (multi-chunk tile blocks + their slab reduce,
 *           the row kernel);  part 0: all (= gcnk_spmm_csr_f32).
 * Part 2 alone uses the workspace.  (R8's X W1: part 1 = the document rows,
 * part 2 = the 50 dense topic rows, whose reduce launch then overlaps the
 * document blocks instead of following them.) */
int gcnk_spmm_csr_f32_part(const void* plan, const int32_t* plan_header,
                           const float* B, int64_t ldb, int32_t F,
                           float* C, int64_t ldc,
                           const float* bias, int32_t epilogue,
                           const uint8_t* drop_mask, int64_t ldm, float drop_scale,
                           float keep_prob, uint64_t seed, uint64_t offset, const uint64_t* rng_base,
                           float* workspace, int64_t workspace_bytes,
                           int32_t* counters, int64_t counter_bytes,
                           int32_t lanes_hint, int32_t part, void* stream);

/* SpMM with a fused dense projection of every finished row:
 *   H = epi(A B)  (stored to C only when C != NULL),   C2[M x P] = H * W[F x P]
 * i.e. layer.py:106,110,182,185 of gc1 followed by layer.py:102 of gc2
 * (support2 = H1 W2) while H1's row is still in registers: the gc2 GEMM
 * launch and, in inference, the H1 round trip through HBM disappear.
 * Supported for plans without dense tile blocks, float4-aligned operands,
 * F <= 256 and P <= 32; otherwise returns GCNK_EUNSUP (callers then run
 * gcnk_spmm_csr_f32 + gcnk_gemm_f32). */
int gcnk_spmm_proj_f32(const void* plan, const int32_t* plan_header,
                       const float* B, int64_t ldb, int32_t F,
                       float* C, int64_t ldc,
                       const float* bias, int32_t epilogue,
                       const uint8_t* drop_mask, int64_t ldm, float drop_scale,
                       float keep_prob, uint64_t seed, uint64_t offset, const uint64_t* rng_base,
                       const float* W, int64_t ldw, int32_t P, float* C2, int64_t ldc2,
                       float* workspace, int64_t workspace_bytes,
                       int32_t* counters, int64_t counter_bytes,
                       int32_t lanes_hint, void* stream);

/* ---------------------------------------------------------------------------
 * fp32 GEMM on MFMA (v_mfma_f32_16x16x4_f32; exact fp32 FMA chains):
 *   C[M x N] = epi( op(A)[M x K] * op(B)[K x N] )
 * op(A) = A (row-major [M x K], lda) or A^T (A stored [K x M], lda) when transA.
 * op(B) = B ([K x N], ldb) or B^T (B stored [N x K], ldb) when transB.
 * Replaces th.spmm(dense H, W) (layer.py:102 in gc2, which ATen lowers to mm)
 * and the dense autograd products H^T g, g W^T.
 * split_k > 1 reduces K in slabs (workspace = split_k*M*N floats) summed in a
 * fixed order by a second pass (bitwise reproducible).
 * ------------------------------------------------------------------------- */
int64_t gcnk_gemm_workspace_bytes(int32_t M, int32_t N, int32_t K, int32_t split_k);
int gcnk_gemm_f32(int32_t transA, int32_t transB, int32_t M, int32_t N, int32_t K,
                  const float* A, int64_t lda, const float* B, int64_t ldb,
                  float* C, int64_t ldc,
                  const float* bias, int32_t epilogue, const float* R, int64_t ldr, float scale,
                  int32_t split_k, float* workspace, int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * out[n] = sum_m X[m, n]  (bias gradient, autograd of layer.py:110).
 * Deterministic two-pass reduction; workspace = gcnk_colsum_workspace_bytes.
 * ------------------------------------------------------------------------- */
int64_t gcnk_colsum_workspace_bytes(int32_t M, int32_t N);
int gcnk_colsum_f32(const float* X, int64_t ldx, int32_t M, int32_t N, float* out,
                    float* workspace, int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Fused backward of gc2 and of gc1's ReLU + dropout (autograd of
 * layer.py:182-188 through layer.py:102-110; replaces gcnk_gemm_f32 with
 * GCNK_GEMM_EPI_MASK_POS for gZ1, the split-K gcnk_gemm_f32 for gW2 and two
 * gcnk_colsum_f32 calls):
 *   gZ1[m, n] = H[m, n] > 0 ? scale * (gS[m, :] . W[n, :]) : 0     [M x N, ldz]
 *   gW[n, p]  = sum_m H[m, n] gS[m, p]                             [N x P, contiguous]
 *   gb1[n]    = sum_m gZ1[m, n]                                    [N]
 *   gb2[p]    = sum_m G[m, p]                 (G nullable)         [P]
 * H = gc1's output after ReLU + dropout [M x N], gS = A^T G [M x P], W = W2
 * [N x P].  gW / gb1 / gb2 are nullable (not stored).  P <= 32 (else
 * GCNK_EUNSUP).  Two launches; sums in a fixed order (bitwise reproducible).
 * Workspace: gcnk_gcn_bwd2_workspace_bytes(M, N, P).
 * ------------------------------------------------------------------------- */
int64_t gcnk_gcn_bwd2_workspace_bytes(int32_t M, int32_t N, int32_t P);
int gcnk_gcn_bwd2_f32(const float* H, int64_t ldh, const float* gS, int64_t ldgs, const float* W, int64_t ldw,
                      const float* G, int64_t ldg, int32_t M, int32_t N, int32_t P, float scale,
                      float* gZ1, int64_t ldz, float* gW, float* gb1, float* gb2,
                      void* workspace, int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Hub-factored gc1 (csrc/factor.hip; GCN.forward layer.py:164-190 through
 * layer.py:102,106,110,182,185 and gc2's support layer.py:102) for a graph
 * whose rows split into hub rows and light rows referencing only hub columns
 * and themselves, with X's light rows inside the column range [k0, k0 + Kc):
 *   Z[r, :]   = U[i, :Kc] . W[k0 .. k0+Kc-1, :] + sum_{items of r} val * S[hub, :]
 *   H[r, n]   = epilogue(Z[r, n] + bias[n])            (GCNK_EPI_*, as the SpMM)
 *   C2[r, p]  = sum_n H[r, n] W2[n, p]                 (P <= 32)
 * for r = the row id at position i of the block order.  U [M x Kc] in block
 * order (ldu >= Kc rounded up to 4, zero past Kc), S = X[hubs] W [nhub x F]
 * (lds), rec = one record of rec_words int32 per 32-row block: 33 offsets
 * (block-relative item index), 3 pad words, 32 row ids (the output rows of the
 * block's positions, -1 past M), then items int2 {hub index, value bits}.  H
 * nullable (not stored).  F % 4 == 0, F <= 256, Kc <= 128; GCNK_EUNSUP when
 * the block's operands exceed 160 KiB of LDS (gcnk_hubfactor_lds_bytes).  One
 * launch, fixed-order sums.
 * ------------------------------------------------------------------------- */
int64_t gcnk_hubfactor_lds_bytes(int32_t F, int32_t Kc, int32_t nhub, int32_t rec_words, int32_t P);
/* Test aid: fills every CU's 160 KiB of LDS with `word` (one launch), so a
 * following launch that read LDS it had not written would see it. */
int gcnk_debug_poison_lds(uint32_t word, void* stream);
int gcnk_hubfactor_gc1_f32(int32_t M, int32_t F, int32_t Kc, int32_t nhub, int32_t P, const float* U, int64_t ldu,
                           const float* W, int64_t ldw, int32_t k0, const float* S, int64_t lds,
                           const int32_t* rec, int32_t rec_words, const float* bias, int32_t epilogue,
                           const uint8_t* drop_mask, int64_t ldm, float drop_scale, float keep_prob, uint64_t seed,
                           uint64_t offset, const uint64_t* rng_base, const float* W2, int64_t ldw2, float* H,
                           int64_t ldh, float* C2, int64_t ldc2, void* stream);
/* ---------------------------------------------------------------------------
 * Narrow-feature gc1 (csrc/dense_gc1.hip; GCN.forward layer.py:164-190 through
 * layer.py:102,106,110,182,185 and gc2's support layer.py:102) for a dense X
 * with at most 128 features (the gensim-shaped topic features, README.md:77,95):
 * with AX = A-hat X [M x K] (ldax >= K, gcnk_aggregate_f32, built once per
 * (A-hat, X) pair),
 *   H[r, n]  = epilogue((AX W1)[r, n] + bias[n])   (GCNK_EPI_BIAS_RELU[_DROP|_HASH])
 *   C2[r, p] = sum_n H[r, n] W2[n, p]
 * in one launch (fp32 MFMA, fixed-order sums).  H nullable (not stored).
 * K <= 128, F <= 256, P <= 32 (GCNK_EUNSUP otherwise).  The association
 * (A-hat X) W1 differs from the reference's A-hat (X W1) in fp32 rounding only.
 *   gcnk_aggregate_f32: out[r, c] = fp32( sum over row r's items in CSR order,
 *   in float64, of val * X[col, c] ), c < K; 0 for K <= c < Kp <= 128.
 * ------------------------------------------------------------------------- */
int gcnk_dense_gc1_f32(int32_t M, int32_t K, int32_t F, int32_t P, const float* AX, int64_t ldax, const float* W1,
                       int64_t ldw1, const float* bias, int32_t epilogue, const uint8_t* drop_mask, int64_t ldm,
                       float drop_scale, float keep_prob, uint64_t seed, uint64_t offset, const uint64_t* rng_base,
                       const float* W2, int64_t ldw2, float* H, int64_t ldh, float* C2, int64_t ldc2, void* stream);
int gcnk_aggregate_f32(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t M, const float* X,
                       int64_t ldx, int32_t K, float* out, int64_t ldo, int32_t Kp, void* stream);

/* The hub factorisation's (A-hat, X)-fixed operands, built on the device once
 * per operand pair (csrc/factor_build.hip; factor.py drives it, the host
 * restatement is oracle/factor_host.py):
 *   gcnk_factor_u_f32:   U[p, c] = fp32( sum over the items (r, d) of row
 *                        r = perm[p], d light (hub_index[d] < 0), in CSR order,
 *                        in float64, of val * Xl[d, c] ), c < Kc; 0 for
 *                        Kc <= c < Kcp <= 128.  Xl [M x >= Kc] (ldxl): X's
 *                        columns k0.. (hub rows never read).
 *   gcnk_factor_records: the per-32-row-block A_H records gcnk_hubfactor_gc1_f32
 *                        reads, into rec [ceil(M/32) x rec_words] (zeroed by
 *                        the call first); *overflow (zeroed by the call)
 *                        counts blocks whose items did not fit.
 *   gcnk_factor_analyze: the structure test in front of them, on the device
 *                        with one host sync (ABI 12; replaces torch element-wise
 *                        / nonzero / index kernels whose first-use loads cost
 *                        the first forward ~120 ms): hub rows = rows of >= hmin
 *                        nonzeros; host outputs info[8] = {H, bad (a light row
 *                        with a column that is neither a hub nor its diagonal),
 *                        k0, k1 (column range of X's nonzero entries in light
 *                        rows, k1 = -1 if none), total length of X's hub rows
 *                        (CSR X), 0, 0, 0}, hubs[max_hubs] (the first H found,
 *                        unordered; H > max_hubs: some missing), cnt[M] (each
 *                        row's hub-column items).  X: CSR (x_rowptr non-NULL, M
 *                        rows) or dense [M x K] (x_dense, ldx).  Workspace:
 *                        gcnk_factor_analyze_workspace_bytes(M, max_hubs).
 *   gcnk_factor_xl_f32:  Xl [M x Kcp] (ldxl) = X[r, k0 .. k0 + Kc) for light
 *                        rows (hub_index[r] < 0) of a CSR X, zero elsewhere.
 *   gcnk_csr_gather_rows / gcnk_dense_gather_rows_f32: the rows `rows[0 ..
 *                        nrows)` of a CSR (out_rowptr[nrows + 1] written; out
 *                        arrays sized by the caller) or of a dense matrix (out
 *                        [nrows x ldo], columns K .. ldo - 1 zero): X's hub rows. */
int gcnk_factor_u_f32(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t M,
                      const int32_t* hub_index, const int32_t* perm, const float* Xl, int64_t ldxl, int32_t Kc,
                      float* U, int64_t ldu, int32_t Kcp, void* stream);
int gcnk_factor_records(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t M,
                        const int32_t* hub_index, const int32_t* perm, int32_t* rec, int32_t rec_words,
                        int32_t* overflow, void* stream);
int64_t gcnk_factor_analyze_workspace_bytes(int32_t M, int32_t max_hubs);
int gcnk_factor_analyze(const int32_t* rowptr, const int32_t* colind, int32_t M, int32_t hmin,
                        const int32_t* x_rowptr, const int32_t* x_colind, const float* x_val,
                        const float* x_dense, int64_t ldx, int32_t K, int32_t max_hubs, int32_t* info /* host */,
                        int32_t* hubs /* host */, int32_t* cnt /* host */, void* workspace, int64_t workspace_bytes,
                        void* stream);
int gcnk_factor_xl_f32(const int32_t* x_rowptr, const int32_t* x_colind, const float* x_val, int32_t M,
                       const int32_t* hub_index, int32_t k0, int32_t Kc, float* Xl, int64_t ldxl, int32_t Kcp,
                       void* stream);
int gcnk_csr_gather_rows(const int32_t* rowptr, const int32_t* colind, const float* val, const int32_t* rows,
                         int32_t nrows, int32_t* out_rowptr, int32_t* out_colind, float* out_val, void* stream);
int gcnk_dense_gather_rows_f32(const float* X, int64_t ldx, int32_t K, const int32_t* rows, int32_t nrows,
                               float* out, int64_t ldo, void* stream);

/* ---------------------------------------------------------------------------
 * Whole-forward launch record (ABI 8): GCN.forward (layer.py:164-190) as the
 * reference's trainer issues it, eagerly, every epoch (trainer.py:357 train,
 * trainer.py:382 eval) -- from ONE call.  The caller fills the record once per
 * (adjacency, features, widths, stream) with everything that does not change
 * from call to call: the plans and their host headers, workspaces and counter
 * regions, the factored operands, the intermediates S1 and S2.  Each call
 * passes only the parameters, the outputs and the dropout arguments, and
 * issues the launches the per-op entry points above issue, in the same order
 * and with the same arguments (results are bitwise those of the per-op path).
 *
 *   GCNK_FWD_FACTORED   S_T = X_hubs W1 (x plan or dense GEMM, x_rows = nhub);
 *                       (H1, S2) = gcnk_hubfactor_gc1_f32; out = A-hat S2 + b2
 *   GCNK_FWD_SPMM_PROJ  S1 = X W1; (H1, S2) = gcnk_spmm_proj_f32(aF); out = A-hat S2 + b2
 *   GCNK_FWD_SPMM_GEMM  S1 = X W1; H1 = epi(A-hat S1 + b1) (aF); S2 = H1 W2; out = A-hat S2 + b2
 *   GCNK_FWD_DENSE_AX   (H1, S2) = gcnk_dense_gc1_f32(U = A-hat X [M x Kc], ldu); out = A-hat S2 + b2
 *                       (no first product: x, s1 unused)
 *
 * gc2's aggregation uses the plan aP with GCNK_EPI_BIAS (GCNK_EPI_NONE when b2
 * is NULL).  W1 [x_cols x F] and W2 [F x P] contiguous; H1 (ldh) is stored
 * when non-NULL (a backward needs it); SPMM_GEMM needs h1_tmp [M x F] when it
 * is NULL.  The record's buffers are used in stream order: calls that may
 * run concurrently need records of their own.
 * ------------------------------------------------------------------------- */
typedef struct gcnk_plan_ref {
  const void* plan;            /* device plan image (gcnk_spmm_plan_build) */
  int32_t hdr[16];             /* its header (gcnk_spmm_plan_query) */
  float* workspace;            /* gcnk_spmm_workspace_bytes(hdr, width) bytes */
  int64_t workspace_bytes;
  int32_t* counters;           /* gcnk_spmm_counter_bytes(hdr) bytes (zeroed once) */
  int64_t counter_bytes;
  int32_t lanes_hint;
  int32_t pad_;
} gcnk_plan_ref;

#define GCNK_FWD_FACTORED 1
#define GCNK_FWD_SPMM_PROJ 2
#define GCNK_FWD_SPMM_GEMM 3
#define GCNK_FWD_DENSE_AX 4

typedef struct gcnk_gcn_fwd {
  int32_t kind;
  int32_t M, F, P;             /* rows of A-hat, nhid, nclass */
  int32_t x_rows, x_cols;      /* first product's operand (factored: the hub rows of X) */
  gcnk_plan_ref x;             /* sparse operand: its plan (x.plan != NULL) ...       */
  const float* x_dense;        /* ... or dense [x_rows x x_cols] (ldx) on the MFMA GEMM */
  int64_t ldx;
  int32_t x_split_k;
  int32_t pad0_;
  float* gemm_ws;              /* GEMM split-K workspace (first product and H1 W2) */
  int64_t gemm_ws_bytes;
  float* s1;                   /* S1 = X W1, or S_T = X_hubs W1 [x_rows x F] */
  int64_t lds1;
  int32_t Kc, nhub, k0, rec_words;   /* factored gc1 (gcnk_hubfactor_gc1_f32); DENSE_AX: Kc = K */
  const float* U;
  int64_t ldu;
  const int32_t* rec;
  gcnk_plan_ref aF;            /* A-hat at width F (SPMM kinds) */
  gcnk_plan_ref aP;            /* A-hat at width P (gc2) */
  float* s2;                   /* S2 = H1 W2 [M x P] */
  int64_t lds2;
  float* h1_tmp;               /* SPMM_GEMM scratch H1 when H1 == NULL */
  int64_t ld_h1_tmp;
} gcnk_gcn_fwd;

int gcnk_gcn_forward_f32(const gcnk_gcn_fwd* rec,
                         const float* W1, const float* b1, const float* W2, const float* b2,
                         float* out, int64_t ldo, float* H1, int64_t ldh,
                         int32_t epilogue, const uint8_t* drop_mask, int64_t ldm, float drop_scale,
                         float keep_prob, uint64_t seed, uint64_t offset, const uint64_t* rng_base,
                         void* stream);
/* The backward of the same forward (trainer.py:361 loss.backward()), from
 * one call, with gcnk_gcn_bwd filled once per (adjacency, features, widths,
 * stream) -- the launches ops.GCNFn.backward issues, in its order:
 *   gS2 = A-hat^T G                          (aTP: A-hat^T's plan at width P)
 *   gZ1, gW2, gb1, gb2 = gcnk_gcn_bwd2_f32(H1, gS2, W2, G)  (bwd2 workspace)
 *   gS1 = A-hat^T gZ1; gW1 = X^T gS1         (aTF; X^T's plan xT, or the MFMA
 *                                             GEMM on dense X with x_split_k)
 * G = dlogits [M x P] (contiguous), H1 [M x F] (ldh), W2 [F x P].  gW1, gb1,
 * gW2, gb2 are nullable (not computed); gb2 needs G's column sums only.
 * flags & GCNK_BWD_AX_DIRECT: x_dense holds A-hat X (the DENSE_AX forward) and
 * gW1 = (A-hat X)^T gZ1 directly (no gS1, no aTF plan).
 * (ABI 11's GCNK_BWD_FACTORED -- gW1 through the hub factor -- measured slower
 * than A-hat^T gZ1 + X^T gS1 in the step and was removed in ABI 12.) */
#define GCNK_BWD_AX_DIRECT 1
typedef struct gcnk_gcn_bwd {
  int32_t M, F, P;             /* rows of A-hat, nhid, nclass */
  int32_t x_rows, x_cols;      /* X [x_rows x x_cols]: gW1 is [x_cols x F] */
  int32_t x_split_k;           /* dense X: K-slabs of X^T gS1 */
  int32_t flags;               /* GCNK_BWD_* */
  int32_t pad1_;
  gcnk_plan_ref aTP, aTF;      /* A-hat^T at widths P and F */
  gcnk_plan_ref xT;            /* sparse X: X^T's plan at width F (xT.plan != NULL) ... */
  const float* x_dense;        /* ... or dense X (ldx) */
  int64_t ldx;
  float* gemm_ws;              /* split-K workspace of X^T gS1 */
  int64_t gemm_ws_bytes;
  float* gS2;                  /* scratch [M x P] */
  float* gZ1;                  /* scratch [M x F] */
  float* gS1;                  /* scratch [M x F] */
  void* bwd2_ws;               /* gcnk_gcn_bwd2_workspace_bytes(M, F, P) */
  int64_t bwd2_ws_bytes;
} gcnk_gcn_bwd;

int gcnk_gcn_backward_f32(const gcnk_gcn_bwd* rec, const float* G, const float* H1, int64_t ldh, const float* W2,
                          float scale, float* gW1, float* gb1, float* gW2, float* gb2, void* stream);

/* Layout of the record structs for bindings that mirror them: writes up to n
 * of {sizeof plan_ref, sizeof gcn_fwd, offsetof x, U, aF, aP, ld_h1_tmp,
 * plan_ref.lanes_hint, sizeof gcn_bwd, gcn_bwd.xT, gcn_bwd.bwd2_ws_bytes} to
 * out and returns how many exist. */
int32_t gcnk_gcn_fwd_layout(int64_t* out, int32_t n);

/* ---------------------------------------------------------------------------
 * Sparse-format helpers (one-time graph preparation, utils.py:185-213,
 * trainer.py:226-238).
 *   gcnk_csr_transpose: CSR A[M x K] -> CSR A^T[K x M]; within each output
 *     row entries keep ascending source-row order (stable).  Needs a
 *     workspace of gcnk_csr_transpose_workspace_bytes.
 * ------------------------------------------------------------------------- */
int64_t gcnk_csr_transpose_workspace_bytes(int32_t M, int32_t K, int64_t nnz);
/*  gcnk_coo_to_csr: the torch sparse COO tensors the reference hands th.spmm
 *    (utils.py:196-203: A-hat column-major and uncoalesced; trainer.py:226-238:
 *    X row-major) -> int32 CSR with sorted columns, duplicates summed in input
 *    order (what ATen's coalesce computes).  rows/cols int64[nnz], vals fp32;
 *    outputs have capacity nnz; rowptr[M] is the output nnz (read it after the
 *    stream completes; -1 if an index was out of range).  Replaces ATen's
 *    coalesce + bincount on the one-time conversion path. */
int64_t gcnk_coo_to_csr_workspace_bytes(int64_t nnz, int32_t M, int32_t K);
int gcnk_coo_to_csr(const int64_t* rows, const int64_t* cols, const float* vals, int64_t nnz, int32_t M, int32_t K,
                    int32_t* rowptr, int32_t* colind, float* val, void* workspace, int64_t workspace_bytes,
                    void* stream);
int gcnk_csr_transpose(const int32_t* rowptr, const int32_t* colind, const float* val,
                       int32_t M, int32_t K, int64_t nnz,
                       int32_t* rowptr_t, int32_t* colind_t, float* val_t,
                       void* workspace, int64_t workspace_bytes, void* stream);
/*  gcnk_csr_to_dense: CSR A[M x K] -> dense row-major out[M x ld] (columns
 *    K..ld-1 untouched; duplicate entries summed in CSR order).  The one-time
 *    layout change that sends a dense-enough sparse infeatn (layer.py:102;
 *    e.g. a gensim-style 100-d X at 50-70 % fill) to the MFMA GEMM. */
int gcnk_csr_to_dense(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t M, int32_t K,
                      float* out, int64_t ld, void* stream);

/* ---------------------------------------------------------------------------
 * Device-side adjacency preparation (utils.py:185-213, preprocess_adj /
 * normalize_adj, which the reference runs on the host with scipy):
 *   A_hat = D^-1/2 (A + I) D^-1/2,  D = rowsum(A + I)
 * with the reference's arithmetic (A + I and D in float64, d = rowsum^-0.5,
 * inf -> 0, value = (d[r] * a) * d[c] rounded once to fp32), so the values are
 * bit-for-bit the reference's.  Input: n x n CSR with sorted, duplicate-free
 * columns per row (a symmetric A, as trainer.py:148 makes it).  Output CSR
 * arrays have capacity nnz + n; rowptr_out[n] is the output nnz (read it
 * after the stream completes).  Workspace: gcnk_sym_normalize_workspace_bytes.
 * ------------------------------------------------------------------------- */
int64_t gcnk_sym_normalize_workspace_bytes(int32_t n, int64_t nnz);
int gcnk_sym_normalize(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t n, int64_t nnz,
                       int32_t* rowptr_out, int32_t* colind_out, float* val_out,
                       void* workspace, int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Evaluation counts in one launch (utils.py:25-109 accuracy / macro_f1 issue
 * 3 * nclass + 1 .item() syncs): for the n scored rows (row = idx[i], or i
 * when idx is NULL) of logits [rows x nclass] (leading dimension ld) with
 * int64 labels `target` (indexed by row), predicted class = first maximal
 * logit (NaN counts as maximal: th.max semantics); counts[3 * nclass + 1]
 * (zeroed by the call) = TP[nclass] | FP[nclass] | FN[nclass] | correct.
 * nclass <= 1024.  Integer atomics: exact.
 * ------------------------------------------------------------------------- */
int gcnk_class_stats(const float* logits, int64_t ld, const int64_t* target, const int64_t* idx, int64_t n,
                     int32_t nclass, int32_t* counts, void* stream);

/* ---------------------------------------------------------------------------
 * Weighted edge-list loader (HOST pointers; no device work): the graph file
 * build_graph.py:199 writes (nx.write_weighted_edgelist: "u v weight" lines,
 * integer node ids) -> the symmetric float32 adjacency trainer.py:98-148
 * builds from it, as an int32 CSR with sorted, duplicate-free columns
 * (a repeated edge keeps its last weight; ids must be 0..n-1).
 * gcnk_edgelist_size gives n and nnz; gcnk_edgelist_csr fills host buffers
 * rowptr[n + 1], colind[nnz], val[nnz].
 * ------------------------------------------------------------------------- */
int gcnk_edgelist_size(const char* path, int64_t* n_nodes, int64_t* nnz);
int gcnk_edgelist_csr(const char* path, int64_t n_nodes, int64_t nnz, int32_t* rowptr, int32_t* colind, float* val);

/* ---------------------------------------------------------------------------
 * Dropout keep-mask exactly as the reference's CPU th.dropout draws it
 * (HOST pointers; layer.py:185 -> ATen dropout -> empty_like(x).bernoulli_(p)
 * with p = 1 - dropout): torch's serial CPU bernoulli_ takes one 64-bit draw
 * of the MT19937 generator per element, in order, and keeps the element when
 * (draw & (2^53 - 1)) * 2^-53 < p.  `state` (624 words), `left` and `next` are
 * the generator's state fields (torch's CPU generator state tensor), advanced
 * in place by the 2 n outputs consumed, so writing them back leaves the
 * process's random stream where the reference leaves it.  mask_out[n]: 1 =
 * kept.  One pass, one thread (the twist chain is serial); `threads` is
 * accepted and ignored.
 * ------------------------------------------------------------------------- */
int gcnk_bernoulli_mt19937(uint32_t* state, int32_t* left, int64_t* next, int64_t n, double p, uint8_t* mask_out,
                           int32_t threads);

/* The same draw on a native worker thread (a training loop draws the next
 * step's mask while the GPU runs this one).  *job receives a handle; the
 * buffers must stay alive and untouched until gcnk_bernoulli_mt19937_wait(job)
 * returns, and every started job is waited for exactly once. */
int gcnk_bernoulli_mt19937_start(uint32_t* state, int32_t* left, int64_t* next, int64_t n, double p,
                                 uint8_t* mask_out, void** job);
int gcnk_bernoulli_mt19937_wait(void* job);

/* Measurement floor (not on the GCN path): dst[0..n) = src[0..n) as one
 * float4 grid-stride launch -- the north-star SpMM's dense bytes with no CSR
 * and no gathers (bench.py's "copy" roofline line). */
int gcnk_stream_copy_f32(const float* src, float* dst, int64_t n, void* stream);

/* Debug only: in a library built with -DGCNK_STAMPS, when `buf` is non-null
 * every later row/tile SpMM launch writes 4 x uint64 s_memrealtime stamps
 * (100 MHz) per workgroup to it (entry, items staged, chunk walked, exit).
 * Process-global and not thread-safe, which is why the product build
 * compiles it out: there it returns GCNK_EUNSUP for a non-null buffer. */
int gcnk_debug_set_stamps(void* buf);

#ifdef __cplusplus
}
#endif

#endif /* GCNK_H_ */
