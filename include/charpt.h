/*
 * charpt -- MI355X-native (gfx950/CDNA4) kernels for the char-level GPT hot path of
 * ChaitIITB/ReplicatingGPT GPT1.py.  C ABI of libcharpt_hip.so.
 *
 * The reference has no native plugin API: its replaceable seam is the nn.Module surface and
 * the aten ops those modules call.  Every entry point below replaces one or
 * more of those aten call sites; the citation on each names the GPT1.py line(s) it stands in
 * for.  Python binds these through ctypes (replicatinggpt_amd/_lib.py) and registers them as
 * torch.library custom ops (replicatinggpt_amd/ops.py).
 *
 * Conventions
 *   - all pointers are DEVICE pointers unless noted; the caller (PyTorch's caching allocator)
 *     owns every buffer; the library never allocates, frees or synchronises the host.
 *   - every function is stream-ordered on `stream` (a hipStream_t, passed as void*), so it is
 *     capturable into a hipGraph.
 *   - state: the library keeps no per-call state except the DEFERRED WORK below and the
 *     cg_set_tuning knobs, which only select kernels / schedules for A/B and test runs (never the
 *     numerics of a call: precision and deferral are per-call flags).
 *   - deferred work (per stream): a call asks for it explicitly -- cg_epilogue_t.flags
 *     CG_GEMM_DEFER_REDUCE (a split-K weight-gradient reduce left pending), cg_adamw_defer, and the
 *     CG_DEFER flag of cg_reduce_rows_ex / cg_layernorm_bwd_reduce_ex / cg_head_bwd_ex (column-sum
 *     reduces queued for one multi-job launch).  The queue is that of the call's stream, keyed by
 *     (the stream's own device, stream) whatever device is current in the calling thread: only a
 *     later persistent GEMM launch on the SAME stream takes its jobs (in its tail / free blocks),
 *     and cg_flush_deferred(stream) launches the rest on that stream, with the stream's device made
 *     current for the launches (the caller's restored).  A flushed or discarded queue is dropped,
 *     so a new stream that reuses a destroyed stream's handle starts with an empty one.  A mutex guards the
 *     queue registry, so host threads that each drive their own stream are safe; two threads
 *     sharing one stream must order their calls themselves, as with any stream.  Until the flush,
 *     the caller keeps every queued job's workspace alive and reads none of its outputs.
 *   - cg_last_error_string() is per thread.
 *   - return CG_OK (0) or an error code; cg_last_error_string() gives the message.
 *   - dtype codes: CG_F32 = 0 (float), CG_BF16 = 1 (bfloat16 bits, RNE rounding).
 *   - dropout: Philox4x32-10 counter RNG, spec in oracle/philox.py and DESIGN.md; the stream id
 *     is ((*rng_call) << 8) | site, with rng_call a device uint64 snapshot per forward call.
 */
#ifndef CHARPT_H
#define CHARPT_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { CG_OK = 0, CG_EINVAL = 1, CG_EHIP = 2, CG_EUNSUPPORTED = 3 };
enum { CG_F32 = 0, CG_BF16 = 1 };
/* cg_epilogue_t.aux_dtype only: ReLU keep bits, uint32 words [M][ld_aux], bit n % 32 of word n / 32
   of row m = (bf16 ReLU output (m, n) != 0).  CG_EPI_BIAS_RELU WRITES them (aux is an output there),
   CG_EPI_RELU_BWD reads them instead of the bf16 ReLU output (1/16 of its bytes).  Only where
   cg_gemm_relu_bits_supported() says so (bf16, split 1, beta 0, N % 64 == 0, persistent kernels);
   elsewhere cg_gemm returns CG_EINVAL. */
enum { CG_BITS = 2 };

/* GEMM epilogues (applied to acc = sum_k A(m,k) B(n,k), per output element (m,n)) */
enum {
    CG_EPI_STORE = 0,        /* out = acc                                                       */
    CG_EPI_BIAS = 1,         /* out = acc + bias[n]                                             */
    CG_EPI_BIAS_RELU = 2,    /* out = relu(acc + bias[n])               (GPT1.py:143-144)       */
    CG_EPI_BIAS_RESID = 3,   /* out = resid[m,n] + acc + bias[n]  (resid NULL: no add; :136,163) */
    CG_EPI_BIAS_DROP_RESID = 4, /* out = resid + dropout(acc + bias)    (GPT1.py:145-146,164)   */
    CG_EPI_RELU_BWD = 5,     /* out = acc * (aux[m,n] > 0)              (ReLU backward, :144)   */
    /* 6 unused.  out = acc (bf16), and the attention backward's delta = rowsum(dO * O) per head from
       the written values: colpart[((m / T) * (N / 64) + n / 64) * T + m % T] = sum over the head's 64
       columns of bf16(acc) * aux[m, n]  (aux = the attention output O, bf16, stride ld_aux;
       T = ld_resid, M % T == 0).  Only where cg_gemm_rowdot_supported() says so.               */
    CG_EPI_STORE_ROWDOT = 7
};

typedef struct {
    int kind;                 /* CG_EPI_*                                                    */
    const float* bias;        /* [N] fp32 or NULL                                            */
    const float* resid;       /* fp32, row stride ld_resid                                   */
    int64_t ld_resid;
    const void* aux;          /* CG_EPI_RELU_BWD: relu output, dtype aux_dtype, stride ld_aux */
    int aux_dtype;
    int64_t ld_aux;
    double dropout_p;         /* CG_EPI_BIAS_DROP_RESID                                      */
    uint64_t seed;
    const uint64_t* rng_call; /* device scalar                                               */
    int site;
    float beta;               /* out = epi(acc) + beta * out   (beta in {0,1}: grad accumulate) */
    float* colpart;           /* CG_EPI_RELU_BWD, bf16, beta 0, split 1 only, and only where the
                                 dispatch takes the 128x128 persistent kernel (else CG_EINVAL):
                                 column sums of each 64-row block of the output (of its bf16-
                                 rounded values, as cg_colsum would see them), [M/64][N] -- the consumer's bias-gradient partials,
                                 folded by cg_reduce_rows.  NULL: none.                     */
    int flags;                /* CG_GEMM_* below; 0 = plain (fp32 slabs, reduce in this call) */
} cg_epilogue_t;

/* cg_epilogue_t.flags -- split-K (split_k > 1) fp32 CG_EPI_STORE outputs (the weight gradients):
   CG_GEMM_SLAB_BF16     each split's partial sum is stored as a bf16 slab (rounded once, 2^-9
                         relative) and the slabs are summed in split order in fp32: half the slab
                         bytes.  Applies where the 128x128 persistent kernel runs the product (bf16
                         operands, vectorisable output); elsewhere the call uses fp32 slabs.
   CG_GEMM_DEFER_REDUCE  the slab reduce may stay pending on the stream's deferral queue (above):
                         the next persistent bf16 GEMM on the stream sums it in its tail, or
                         cg_flush_deferred(stream).  Keep the workspace alive until then.  Calls the
                         deferral does not apply to (slab sets > 40 MB) reduce now.                */
enum { CG_GEMM_SLAB_BF16 = 1, CG_GEMM_DEFER_REDUCE = 2 };
/* flags of the _ex column-sum reduces: queue on the stream's deferral queue instead of launching */
enum { CG_DEFER = 1 };

const char* cg_last_error_string(void);
int cg_version(void);
/* process-wide A/B and test knobs (kernel / schedule selection, never a call's numerics): e.g.
   "gemm_variant" 0 = automatic, 2 = register-staged, 9 = persistent 128x128, 24 = 8-wave 256x256,
   97 / 98 = fp32 small-M chunked kernel / 128x64 kernel only, 99 = generic; "decode_attn_rows",
   "red_side", "adam_per_launch", "gemm_n96", "ln_nt", ... (gemm.hip cg_set_tuning).
   Set them before the calls they affect, from one thread.                                       */
int cg_set_tuning(const char* key, int value);
int cg_device_info(int* n_cu, int* arch_major, int* arch_minor);
/* measurement (bench.py's in-step roofline): a timing event recorded on `stream` -- inside a
   hipGraph capture as an EXTERNAL event-record node (hipEventRecordExternal), so that each replay
   re-records it and two such events time the kernels captured between them on that stream.
   cg_timing_event_elapsed: milliseconds between two recorded events (after they completed).     */
int cg_timing_event_create(void** event);
int cg_timing_event_record(void* event, void* stream);
int cg_timing_event_elapsed(void* start, void* end, float* ms);
int cg_timing_event_destroy(void* event);

/* ---- utility ------------------------------------------------------------------------ */
/* *counter += delta (one thread); snapshot variant: *snap = *counter, *counter += 1.       */
int cg_counter_add(int64_t* counter, int64_t delta, void* stream);
int cg_rng_snapshot(uint64_t* counter, uint64_t* snap, void* stream);
/* dst[i] = dropout keep-mask (1.0 / 0.0) for element i in [0,n), for tests of the RNG.    */
int cg_dropout_mask(float* dst, int64_t n, double p, uint64_t seed, const uint64_t* rng_call, int site,
                    void* stream);
/* y[r,c] = x[r,c] * keep(r*C+c) * 1/(1-p)  (dropout backward / apply; p=0 -> plain cast);
   x fp32 [rows, C] (row stride ldx), y dtype y_dtype [rows, C] contiguous.                  */
int cg_dropout_apply(const float* x, int64_t rows, int64_t C, int64_t ldx, void* y, int y_dtype, double p,
                     uint64_t seed, const uint64_t* rng_call, int site, void* stream);
/* deterministic sum of n floats into *out (two-pass); ws >= 1024 floats; out = scale*sum   */
int cg_sum_f32(const float* x, int64_t n, float scale, float* out, float* ws, void* stream);
/* fp32 -> bf16 cast (RNE), n elements                                                       */
int cg_cast_f32_bf16(const float* x, uint16_t* y, int64_t n, void* stream);

/* ---- data: get_batch on device (GPT1.py:75-83) ---------------------------------------- */
/* x[b,t] = data[ix[b]+t], y[b,t] = data[ix[b]+t+1]; data is the token stream (int64 or uint8) */
int cg_gather_batch(const void* data, int data_is_u8, const int64_t* ix, int64_t* x, int64_t* y,
                    int64_t B, int64_t T, void* stream);

/* ---- embeddings (GPT1.py:179-181) ------------------------------------------------------ */
/* x[b,t,:] = wte[idx[b,t],:] + wpe[t,:]  (fp32)                                          */
int cg_embed_fwd(const int64_t* idx, const float* wte, const float* wpe, float* x, int64_t B, int64_t T,
                 int64_t C, int64_t V, void* stream);
/* dwte[v,:] (=|+=) sum_{idx=v} dx ; dwpe[t,:] (=|+=) sum_b dx[b,t,:]   deterministic.
   workspace: cg_embed_bwd_workspace(B,T,C,V) bytes.                                          */
int64_t cg_embed_bwd_workspace(int64_t B, int64_t T, int64_t C, int64_t V);
int cg_embed_bwd(const int64_t* idx, const float* dx, float* dwte, float* dwpe, int64_t B, int64_t T,
                 int64_t C, int64_t V, int accumulate, void* workspace, void* stream);

/* ---- LayerNorm (nn.LayerNorm, GPT1.py:159-160,173) -------------------------------------- */
/* y = (x-mu)*rstd*w + b, biased variance, eps; y dtype y_dtype; saves mean/rstd [rows]     */
int cg_layernorm_fwd(const float* x, const float* w, const float* b, void* y, int y_dtype, float* mean,
                     float* rstd, int64_t rows, int64_t C, float eps, void* stream);
/* dx = dres + LN'(dy)  (dres may be NULL); dx_bf16 optional bf16 copy of dx;
   dw/db (=|+=) column sums; workspace: cg_layernorm_bwd_workspace(rows,C) bytes.           */
int64_t cg_layernorm_bwd_workspace(int64_t rows, int64_t C);
int cg_layernorm_bwd(const void* dy, int dy_dtype, const float* x, const float* w, const float* mean,
                     const float* rstd, const float* dres, float* dx, uint16_t* dx_bf16, float* dw, float* db,
                     int accumulate, void* workspace, int64_t rows, int64_t C, void* stream);
/* the same, with the consumer-side extras: lp_out = bf16(keep ? dx / (1 - p) : 0) (keep from the
   Philox stream (lp_seed, lp_rng_call, lp_site), element idx = r*C + c; p = 0: plain bf16 copy) and
   lp_colsum (+)= column sums of that tensor (fp32, before rounding).                              */
int cg_layernorm_bwd_ex(const void* dy, int dy_dtype, const float* x, const float* w, const float* mean,
                        const float* rstd, const float* dres, float* dx, uint16_t* lp_out, double lp_dropout_p,
                        uint64_t lp_seed, const uint64_t* lp_rng_call, int lp_site, float* dw, float* db,
                        float* lp_colsum, int accumulate, int colsum_accumulate, void* workspace, int64_t rows,
                        int64_t C, void* stream);
/* cg_layernorm_bwd_ex in two launches, so the column-sum reduce can run off the critical path:
   _rows writes dx / lp_out and leaves the per-block column partials (dw, db, and with lp_colsum=1
   the lp_out column sums) in the workspace; _reduce (any stream ordered after _rows) folds them
   into dw / db / lp_colsum exactly as cg_layernorm_bwd_ex does (same order, same bits).       */
int cg_layernorm_bwd_rows(const void* dy, int dy_dtype, const float* x, const float* w, const float* mean,
                          const float* rstd, const float* dres, float* dx, uint16_t* lp_out, double lp_dropout_p,
                          uint64_t lp_seed, const uint64_t* lp_rng_call, int lp_site, int lp_colsum,
                          void* workspace, int64_t rows, int64_t C, void* stream);
int cg_layernorm_bwd_reduce(const void* workspace, int64_t rows, int64_t C, int lp_colsum_partials, float* dw,
                            float* db, float* lp_colsum, int accumulate, int colsum_accumulate, void* stream);
/* the same with flags: CG_DEFER queues the reduce on the stream's deferral queue                */
int cg_layernorm_bwd_reduce_ex(const void* workspace, int64_t rows, int64_t C, int lp_colsum_partials, float* dw,
                               float* db, float* lp_colsum, int accumulate, int colsum_accumulate, int flags,
                               void* stream);

/* ---- GEMM (nn.Linear fwd/dgrad/wgrad: GPT1.py:111-112,121,136,143,145,184) -------------
   C[m,n] = epilogue( sum_k A(m,k) * B(n,k) )
   A(m,k) = A[m*lda+k] (a_trans=0) or A[k*lda+m] (a_trans=1); same for B with b_trans.
   op_dtype: CG_BF16 (bf16 MFMA, fp32 accumulate) or CG_F32 (exact-f32 MFMA).
   c_dtype: output dtype.  split_k > 1 (CG_EPI_STORE/BIAS only) needs workspace of
   cg_gemm_workspace(M,N,split_k) bytes; results are deterministic for any split_k.            */
int64_t cg_gemm_workspace(int64_t M, int64_t N, int split_k);
/* 1 if cg_gemm (bf16, split_k 1, CG_EPI_RELU_BWD with bf16 aux, beta 0) can fill epi->colpart for
   this problem under the current dispatch and tuning knobs (16-B aligned operands assumed), else 0
   -- the caller then computes the bias gradient with cg_colsum instead.                          */
int cg_gemm_colpart_supported(int a_trans, int b_trans, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                              int64_t ldc);
/* 1 if cg_gemm can write (CG_EPI_BIAS_RELU) and read (CG_EPI_RELU_BWD) CG_BITS ReLU keep bits for
   this non-transposed-A bf16 problem (split 1, beta 0) under the current dispatch, else 0.  The
   FeedForward uses them when both its W1 forward and its W2 dgrad products say yes.           */
int cg_gemm_relu_bits_supported(int a_trans, int b_trans, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                                int64_t ldc);
/* 1 if cg_gemm can run CG_EPI_STORE_ROWDOT (bf16 output, split 1, beta 0, N % 64 == 0) for this
   problem under the current dispatch, else 0 -- the attention backward then computes delta itself. */
int cg_gemm_rowdot_supported(int a_trans, int b_trans, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                             int64_t ldc);
/* launch everything still pending on `stream`'s deferral queue (split-K reduces, AdamW jobs, the
   queued column-sum reduces as one launch) on that stream; call it before reading the outputs.
   Same summation order as the in-call forms, so the same bits.                                  */
int cg_flush_deferred(void* stream);
/* drop everything pending on `stream`'s queue without launching it (a failed backward: its
   gradients are abandoned).  *adam_jobs_taken (may be NULL) = the AdamW jobs GEMM launches
   already took from this queue since its last flush / discard -- updates that have run or will
   run; 0 means no parameter has been touched.                                                   */
int cg_discard_deferred(void* stream, int* adam_jobs_taken);
/* out[n] (=|+=) sum_r part[r*N + n] over rows r in order (fixed order: deterministic)          */
int cg_reduce_rows(const float* part, int64_t rows, int64_t N, float* out, int accumulate, void* stream);
int cg_reduce_rows_ex(const float* part, int64_t rows, int64_t N, float* out, int accumulate, int flags,
                      void* stream);
int cg_gemm(int op_dtype, int a_trans, int b_trans, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
            const void* B, int64_t ldb, void* C, int c_dtype, int64_t ldc, const cg_epilogue_t* epi, int split_k,
            void* workspace, void* stream);
/* A residual-stream GEMM with the LayerNorm that reads its output, in one launch (the attention
   projection + ln2, the FFN's second Linear + the next block's ln1 / ln_f: GPT1.py:136,145-147,
   159-160,163-164,173): out = resid + [dropout](A W^T + bias) (fp32; epi kind CG_EPI_BIAS_RESID or
   CG_EPI_BIAS_DROP_RESID with bias and resid, beta 0, flags 0), and y = LN(out; ln_w, ln_b) (bf16,
   row stride N), mean, rstd -- bit for bit cg_gemm followed by cg_layernorm_fwd.  A [M][K] and
   W [N][K] bf16 (lda, ldw), 16-B aligned operands.  Only where
   cg_gemm_resid_layernorm_supported(M, N, K) says 1 (N == 384, M % 64 == 0, K % 64 == 0);
   otherwise CG_EINVAL.                                                                         */
int cg_gemm_resid_layernorm_supported(int64_t M, int64_t N, int64_t K);
int cg_gemm_resid_layernorm(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda, const void* W, int64_t ldw,
                            float* out, int64_t ldc, const cg_epilogue_t* epi, const float* ln_w, const float* ln_b,
                            void* y, float* mean, float* rstd, float eps, void* stream);
/* A Linear over rows of K <= 128 for inference, fp32, optionally with the LayerNorm before it in the
   same launch: out = [resid +] act(a' W^T [+ bias]), a' = LayerNorm(a; ln_w, ln_b, eps) (ln_w, ln_b
   non-NULL: the block's ln1 before the QKV product, GPT1.py:111-112,163; ln2 before FFN1, lnf before
   lm_head) or a' = a; act = relu when relu != 0 (needs bias, no resid); a [M][K] (lda), W [N][K]
   (ldw), resid / out [M][N] (ldr / ldo) -- bit for bit [cg_layernorm_fwd +] cg_gemm (fp32,
   CG_EPI_STORE / CG_EPI_BIAS / CG_EPI_BIAS_RELU / CG_EPI_BIAS_RESID), without the normalised rows in
   memory.  Only where cg_linear_rows_f32_supported(M, N, K) says 1 (K <= 128 even; above 2048 rows
   N <= 2048 even); lda / ldw even and a / W 8-B aligned; above 2048 rows also ldo / ldr even, out /
   resid 8-B aligned and, with the LayerNorm, ln_w / ln_b 8-B aligned and lda == K; else CG_EINVAL. */
int cg_linear_rows_f32_supported(int64_t M, int64_t N, int64_t K);
int cg_linear_rows_f32(int64_t M, int64_t N, int64_t K, const float* a, int64_t lda, const float* ln_w,
                       const float* ln_b, float eps, const float* w, int64_t ldw, const float* bias, int relu,
                       const float* resid, int64_t ldr, float* out, int64_t ldo, void* stream);
/* generate()'s per-token ln1 + QKV product + K/V cache append (GPT1.py:111-113,163 for the newest
   token of each row; the decode engine's phase 1), fp32, one launch: qkv = LayerNorm(x; ln_w, ln_b,
   eps) W^T (x [B][C] (ldx), W [3C][C] (ldw), qkv [B][3C] (ldq)), and columns C..3C-1 of row b also
   to kcache / vcache [B][H][Tmax][C/H] at position *len_dev - 1 -- bit for bit cg_linear_rows_f32
   (with the LayerNorm) then cg_decode_kv_append(qkv, ldq, C, 2C, ...).  B <= 2048, C <= 128 even,
   H | C, ldx / ldw even, x / W 8-B aligned; else CG_EINVAL.                                      */
int cg_decode_qkv_f32(int64_t B, int64_t C, int64_t H, const float* x, int64_t ldx, const float* ln_w,
                      const float* ln_b, float eps, const float* w, int64_t ldw, float* qkv, int64_t ldq,
                      const int64_t* len_dev, int64_t Tmax, float* kcache, float* vcache, void* stream);
/* The FeedForward sublayer's forward for inference (GPT1.py:142-147,164 in eval, no dropout), fp32,
   in one launch: out = resid + (relu(a' W1^T + b1) W2^T + b2) with a' = LayerNorm(a; ln_w, ln_b,
   eps) (ln_w, ln_b non-NULL: the block's ln2, GPT1.py:164) or a' = a (both NULL); a [M][C] (lda),
   W1 [H][C] (ldw1), W2 [C][H] (ldw2), resid / out [M][C] (ldr / ldo; out may alias resid) -- bit for
   bit cg_layernorm_fwd, cg_gemm (fp32, CG_EPI_BIAS_RELU) into an [M][H] buffer and cg_gemm
   (CG_EPI_BIAS_RESID), without the normalised rows or the hidden activations in memory.  Only where
   cg_ffn_fwd_f32_supported(M, C, H) says 1 (C <= 128 even, H <= 2048 even); lda / ldw1 / ldw2 even,
   a / W1 / W2 8-B aligned (with the LayerNorm also ln_w / ln_b, and lda == C); else CG_EINVAL.  (Replaces, in generate()'s window, FeedForward.net's
   two Linear calls and the ln2 before them.)                                                    */
int cg_ffn_fwd_f32_supported(int64_t M, int64_t C, int64_t H);
int cg_ffn_fwd_f32(int64_t M, int64_t C, int64_t H, const float* a, int64_t lda, const float* ln_w, const float* ln_b,
                   float eps, const float* w1, int64_t ldw1, const float* b1, const float* w2, int64_t ldw2,
                   const float* b2, const float* resid, int64_t ldr, float* out, int64_t ldo, void* stream);
/* column sums of a [rows, N] matrix (bias gradients): out[n] (=|+=) sum_m X[m,n]            */
int64_t cg_colsum_workspace(int64_t rows, int64_t N);
int cg_colsum(const void* X, int x_dtype, int64_t rows, int64_t N, int64_t ldx, float* out, int accumulate,
              void* workspace, void* stream);

/* ---- causal self-attention, all heads (Head.forward GPT1.py:109-123 x n_head, :135) -------
   q/k/v element (b,t,h,e) at ptr[(b*T+t)*ld_qkv + h*D + e]; o at o[(b*T+t)*ld_o + h*D + e].
   P = softmax(mask(q k^T * scale)); P = dropout(P); o = P v.  lse[b,h,t] (fp32) saved.      */
int cg_attn_fwd(int dtype, int64_t B, int64_t T, int64_t H, int64_t D, const void* q, const void* k,
                const void* v, int64_t ld_qkv, void* o, int64_t ld_o, float* lse, float scale, double dropout_p,
                uint64_t seed, const uint64_t* rng_call, int site, uint64_t* mask, void* stream);
/* the same with the keep bits already in `mask` (cg_attn_dropmask, e.g. launched ahead on another
   stream so the Philox work overlaps earlier kernels); identical results to cg_attn_fwd.        */
int cg_attn_fwd_premasked(int dtype, int64_t B, int64_t T, int64_t H, int64_t D, const void* q, const void* k,
                          const void* v, int64_t ld_qkv, void* o, int64_t ld_o, float* lse, float scale,
                          double dropout_p, uint64_t seed, const uint64_t* rng_call, int site, uint64_t* mask,
                          void* stream);
/* fill the MFMA path's keep-bit buffer for one attention call (0 < p < 1, T % 64 == 0)          */
int cg_attn_dropmask(int64_t B, int64_t H, int64_t T, double dropout_p, uint64_t seed, const uint64_t* rng_call,
                     int site, uint64_t* mask, void* stream);
/* one launch for a sublayer's LayerNorm forward (cg_layernorm_fwd arguments, GPT1.py:163 ln1) and
   the keep bits of the attention it feeds (cg_attn_dropmask arguments): the two are independent and
   the launch runs them side by side on the CUs (Philox VALU work under the LayerNorm's memory time).
   Results identical to cg_layernorm_fwd followed by cg_attn_dropmask; shapes without a fused form
   (y not bf16, C not 384 / 768, unaligned) take those two launches.                             */
int cg_layernorm_fwd_attn_dropmask(const float* x, const float* w, const float* b, void* y, int y_dtype, float* mean,
                                   float* rstd, int64_t rows, int64_t C, float eps, int64_t B, int64_t H, int64_t T,
                                   double dropout_p, uint64_t seed, const uint64_t* rng_call, int site,
                                   uint64_t* mask, void* stream);
/* keep-bit buffer for dropout on the MFMA (bf16, head_size 64) path: the forward fills it from the
   Philox stream (cg_attn_fwd `mask`, may be NULL on the generic path or with p = 0) and the
   backward reads it (cg_attn_bwd `mask`; NULL -> regenerated inside the workspace).  Layout
   (attention_common.h): per (b*H + h), T/32 + (T/32 - 1)^2/4 tiles of 64 x 32-bit lane words in
   each of two orientations (query-major for the forward / dQ, key-major for dK/dV).            */
int64_t cg_attn_mask_bytes(int64_t B, int64_t H, int64_t T);
/* dq/dk/dv written (not accumulated) with stride ld_dqkv; workspace cg_attn_bwd_workspace. */
int64_t cg_attn_bwd_workspace(int64_t B, int64_t T, int64_t H, int64_t D);
int cg_attn_bwd(int dtype, int64_t B, int64_t T, int64_t H, int64_t D, const void* q, const void* k,
                const void* v, int64_t ld_qkv, const void* o, int64_t ld_o, const void* dout, int64_t ld_do,
                const float* lse, void* dq, void* dk, void* dv, int64_t ld_dqkv, float scale, double dropout_p,
                uint64_t seed, const uint64_t* rng_call, int site, const uint64_t* mask, void* workspace,
                void* stream);
/* cg_attn_bwd with delta = rowsum(dO * O) already computed (fp32 [B][H][T], e.g. by the dO GEMM's
   CG_EPI_STORE_ROWDOT epilogue); the sequence-resident kernels (T <= 256) read it instead of
   loading O, other paths recompute it in the workspace.  NULL delta: exactly cg_attn_bwd.         */
int cg_attn_bwd_delta(int dtype, int64_t B, int64_t T, int64_t H, int64_t D, const void* q, const void* k,
                      const void* v, int64_t ld_qkv, const void* o, int64_t ld_o, const void* dout, int64_t ld_do,
                      const float* lse, const float* delta, void* dq, void* dk, void* dv, int64_t ld_dqkv,
                      float scale, double dropout_p, uint64_t seed, const uint64_t* rng_call, int site,
                      const uint64_t* mask, void* workspace, void* stream);

/* ---- cross entropy over the char vocabulary (F.cross_entropy, GPT1.py:189-192) ----------
   logits fp32 [rows, V] (row stride ld); loss_rows[r] = lse_r - logit[r, tgt_r]; lse saved.
   bwd: dlogits = (*g) * g_mult * (softmax - onehot)   (g = dLoss, g_mult = 1/rows).                    */
int cg_ce_fwd(const float* logits, int64_t rows, int64_t V, int64_t ld, const int64_t* targets, float* loss_rows,
              float* lse, void* stream);
int cg_ce_bwd(const float* logits, int64_t rows, int64_t V, int64_t ld, const int64_t* targets, const float* lse,
              const float* g, float g_mult, float* dlogits, int64_t ld_d, void* dst_lp /* optional bf16 copy */,
              void* stream);

/* ---- fused LM head for the bf16 path (ln_f output -> lm_head -> cross entropy, GPT1.py:174,183-192)
   a bf16 [M, C]; wpad bf16 [wpad_rows, C] = lm_head.weight with zero rows V..wpad_rows-1
   (wpad_rows >= 16*ceil(V/16), V <= 128, M % 16 == 0, C % 32 == 0); bias fp32 [V].
   fwd: logits fp32 [M, V] = a wpad^T + b, lse [M]; with targets also *loss = mean CE (workspace
   cg_head_workspace).  bwd: dl bf16 [M, ld_dl] = (*g_loss) g_mult (softmax - onehot) [+ g_logits],
   zero in columns V..ld_dl-1 (the K-padded operand of the dgrad/wgrad GEMMs); db (+)= colsum(dl). */
int64_t cg_head_workspace(int64_t M, int64_t V);
int cg_head_fwd(const void* a, const void* wpad, int64_t wpad_rows, const float* bias, const int64_t* targets,
                float* logits, float* lse, float* loss, void* workspace, int64_t M, int64_t C, int64_t V,
                void* stream);
int cg_head_bwd(const float* logits, const float* lse, const int64_t* targets, const float* g_loss, float g_mult,
                const float* g_logits, void* dl, int64_t ld_dl, float* db, int db_accumulate, void* workspace,
                int64_t M, int64_t V, void* stream);
/* the same with flags: CG_DEFER queues the db column-sum reduce on the stream's deferral queue  */
int cg_head_bwd_ex(const float* logits, const float* lse, const int64_t* targets, const float* g_loss, float g_mult,
                   const float* g_logits, void* dl, int64_t ld_dl, float* db, int db_accumulate, void* workspace,
                   int64_t M, int64_t V, int flags, void* stream);

/* ---- batched decode for generate() (GPT1.py:196-212; replicatinggpt_amd/decode.py) ----------
   len_dev: device int64 = current sequence length (tokens in idx rows, row stride ld).          */
/* out[b, j] = idx[b, max(0, len - T) + j]: the cropped context of GPT1.py:200                   */
int cg_decode_window(const int64_t* idx, int64_t ld, int64_t B, int64_t T, const int64_t* len_dev, int64_t* out,
                     void* stream);
/* x[b] = wte[idx[b, len-1]] + wpe[len-1]  (fp32, the newest token)                              */
int cg_decode_embed(const int64_t* idx, int64_t ld, const float* wte, const float* wpe, int64_t C,
                    const int64_t* len_dev, float* x, int64_t B, void* stream);
/* K/V cache [B, H, Tmax, D] row len-1 <- qkv rows (k / v at column offsets k_off / v_off)        */
int cg_decode_kv_append(const float* qkv, int64_t ld, int64_t k_off, int64_t v_off, int64_t B, int64_t H,
                        int64_t D, int64_t Tmax, const int64_t* len_dev, float* kcache, float* vcache,
                        void* stream);
/* one query per (b, h) against keys 0..n-1 (n = *len_dev, or nkeys when len_dev is NULL; any n
   >= 1: online softmax over 16-key chunks); K/V element (b, h, j, e) at base + b*sb + h*sh + j*sj
   + e; o[b, h*D + e]; D <= 64                                                                    */
int cg_decode_attn(const float* q, int64_t ldq, const float* k, const float* v, int64_t sb, int64_t sh, int64_t sj,
                   int64_t B, int64_t H, int64_t D, const int64_t* len_dev, int64_t nkeys, float scale, float* o,
                   int64_t ldo, void* stream);
/* idx[b, len] <- argmax(logits[b]) (greedy, first index on ties) or an inverse-CDF draw from
   softmax(logits[b]) with u from Philox(*seed_dev, stream = len, counter = b)                     */
int cg_decode_sample(const float* logits, int64_t ldl, int64_t V, int64_t B, int greedy, const uint64_t* seed_dev,
                     const int64_t* len_dev, int64_t* idx, int64_t ld, void* stream);

/* ---- fused AdamW over a flat fp32 buffer (torch.optim.AdamW, GPT1.py:218,233) ------------
   step_ptr: device int64 step count (already incremented for this step).
   p_bf16: optional bf16 shadow written after the update (GEMM operands).                    */
int cg_adamw(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, int64_t n, double lr, double beta1,
             double beta2, double eps, double weight_decay, const int64_t* step_ptr, void* stream);
/* the same update for [0, n) of one region, deferred on `stream`'s queue: run by the free blocks of
   the next persistent GEMM launch on `stream` that has >= 64 of them (a part-filling launch; at most 4 jobs per launch,
   oldest first), else by cg_flush_deferred -- the jobs left, when they are slices of one set of
   buffers, as one segmented launch -- same bits either way.  The gradient must be final in stream order (a
   pending split-K reduce or queued column-sum reduce writing into g is launched first) and nothing launched before the flush may
   read p / p_bf16 / m / v.  n % 4 == 0, p, g, m, v 16-B and p_bf16 8-B aligned. */
int cg_adamw_defer(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, int64_t n, double lr,
                   double beta1, double beta2, double eps, double weight_decay, const int64_t* step_ptr,
                   void* stream);
/* cg_adamw over a host list of nseg (start, length) element segments of the same flat buffers
   (multiples of 4, at most 64): the parameters a step did not defer.  Same bits as cg_adamw. */
int cg_adamw_segments(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, const int64_t* segs, int nseg,
                      double lr, double beta1, double beta2, double eps, double weight_decay,
                      const int64_t* step_ptr, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CHARPT_H */
