/*
 * pg_directgcn.h -- C ABI of the MI355X (gfx950) DirectGCN message-passing hot path.
 *
 * Replaces, per DirectGCN layer, the six PyG `MessagePassing.propagate` calls and the six
 * `nn.Linear` calls of the reference (`src/models/protgram_directgcn.py:101-112`, propagate =
 * gather x[ei[0]] * w -> scatter_add into ei[1], `:137-140` + PyG aggr='add' at `:27`), plus the
 * gate/bias/constant combine (`:116-133`), the model's residual + leaky_relu (`:214-215`) and the
 * propagation-matrix normalisation (`src/utils/graph_utils.py:160-273`) in fused form.
 *
 * Conventions
 *  - Every pointer is DEVICE memory owned by the caller. The library never allocates or frees.
 *  - Every call enqueues work on `stream` (a hipStream_t passed as void*; NULL = legacy default
 *    stream) and returns without synchronising. Calls are stateless and re-entrant.
 *  - Return value: PG_OK (0) or a negative PG_ERR_*; `pg_last_error()` gives a thread-local message.
 *  - Sparse matrices are CSR keyed by DESTINATION row (the reference's ei[1]); `col` is the
 *    SOURCE node (ei[0]). Within a row, entries are sorted by ascending col: this is the order in
 *    which the reference's coalesced COO feeds scatter_add_, so accumulation order matches it.
 *  - Dense matrices are row-major fp32 with an explicit leading dimension (in elements).
 */
#ifndef PG_DIRECTGCN_H
#define PG_DIRECTGCN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PG_ABI_VERSION 4  /* 2: pg_layer_args_t gained drop_p / drop_seed (fused layer dropout); 3: pg_adam_f32 hyper;
                             4: pg_adam_desc_t gained gtype (bf16 gradients) */

#define PG_OK 0
#define PG_ERR_ARG (-1)
#define PG_ERR_HIP (-2)
#define PG_ERR_UNSUPPORTED (-3)

/* Shared-pattern edge record, precomputed weights: one 16-byte load per pattern entry. The three
 * weights are the values of mathcal_A_in, mathcal_A_out and A_undirected_norm at (col -> row)
 * (graph_utils.py:275-287, :160-196). Absent weights (edge_weight=None) are stored as 1.0f. */
typedef struct pg_edge3 {
    int32_t col;
    float w_in;
    float w_out;
    float w_und;
} pg_edge3_t;

/* Shared-pattern edge record, raw counts (fused-normalisation mode). For destination row i and
 * source j = col: a_fwd = count of transition j->i (A_out_w[j,i]), a_bwd = count of i->j,
 * m_und = multiplicity of the undirected entry (2 on a raw self-loop: PyG add_self_loops appends
 * a second loop, graph_utils.py:180; else 1). a_fwd = a_bwd = 0 marks an identity-only diagonal. */
typedef struct pg_edgeraw {
    int32_t col;
    float a_fwd;
    float a_bwd;
    float m_und;
} pg_edgeraw_t;

/* Single-adjacency edge record (non-shared patterns, e.g. gnn_benchmarker.py:297-305 wiring). */
typedef struct pg_edge1 {
    int32_t col;
    float w;
} pg_edge1_t;

/* Per-node normalisation terms for fused mode, float4 per node:
 *   x = 1/rowsum(A_out_w) (0 if the row is empty)   -- graph_utils.py:231-235 on A_out_w
 *   y = 1/rowsum(A_in_w)  (0 if empty)              -- same on A_in_w = A_out_w^T
 *   z = deg_und^-1/2 (0 if deg 0)                    -- graph_utils.py:187-189
 *   w = 0 (padding) */

/* Flags (bit field) accepted by the SpMM entry points. */
#define PG_FLAG_NO_XCD_REMAP (1u << 0) /* keep hardware blockIdx order instead of XCD-contiguous rows */
#define PG_FLAG_EDGE_LDS (1u << 1)     /* stage edge records through LDS (variant B) */
#define PG_FLAG_UNROLL4 (1u << 2)      /* alternate gathers-in-flight depth (variants A/B: 4 instead of 8; C: 8 instead of 4) */
/* SpMM variants: C (default) = per-row-group LDS record window; A = every lane loads the record
 * (PG_FLAG_BCAST_RECORDS); B = block-wide LDS staging of records (PG_FLAG_EDGE_LDS). */
#define PG_FLAG_BCAST_RECORDS (1u << 7) /* SpMM variant A: every lane of a row group loads the record */
/* 4x4-block transposed n-gram kernels (pg_spmm3t_ngram_*): features per lane (the column pieces of a plan block go to
 * the waves of one workgroup; same bits in every variant). Default: 2 for bf16 at F = 256, F / 64 otherwise. */
#define PG_FLAG_NGRAMT_WIDE (1u << 8)   /* F / 64 features per lane (one wave per plan block) */
#define PG_FLAG_NGRAMT_HALVES (1u << 4) /* F / 128 features per lane (two 64 * (F / 128)-feature halves), F >= 128 */
#define PG_FLAG_NGRAMT_NARROW (1u << 3) /* 1 feature per lane (F / 64 pieces of 64 features) */
#define PG_FLAG_DENSE_PREGATED (1u << 14) /* dense kernels: Z from pg_spmm3_gated_f32 (segments already gated) */
#define PG_FLAG_DENSE_TILED (1u << 15)    /* dense forward: the tiled fp32 kernel even where the split-bf16 W-stationary
                                            kernels apply (F_out = 128, K = 384 or 256, no row map: the default) */
#define PG_FLAG_DENSE_X3 (1u << 16)       /* dense forward: the split-bf16 W-stationary kernel (see pg_dense.hip); the
                                             backward ignores it since round 5 (its split-bf16 weight gradient is the
                                             default, PG_FLAG_WGRAD_F32MFMA opts out) */
#define PG_FLAG_WGRAD_BF16_TILED (1u << 11) /* bf16 dense backward: the 128 x 128-tile weight-gradient kernel instead of
                                               the staged 128 x 384 one (default where F_in, F_out % 128 == 0) */
#define PG_FLAG_DGRAD_BF16_TILED (1u << 10) /* bf16 dense backward: the input-gradient kernel that recomputes dpre per
                                               128-column n-tile instead of the resident-A one (default where
                                               F_out <= 256, F_out % 64 == 0 and M >= 256 rows per CU; bit-identical
                                               results) */
#define PG_FLAG_DGRAD_BF16_RESIDENT (1u << 9) /* bf16 dense backward: the resident-A input-gradient kernel at any M its
                                                 F_out takes (below 256 rows per CU its 64-row workgroups underfill
                                                 the GPU, so the default there is the per-n-tile kernel) */
#define PG_FLAG_WGRAD_F32MFMA (1u << 18)  /* fp32 dense backward: the fp32-MFMA weight-gradient kernel instead of the
                                             split-bf16 one (default where F_in % 128 == 0, F_out % 128 == 0 and no
                                             projected residual) */
#define PG_FLAG_DGRAD_F32MFMA (1u << 17)  /* fp32 dense backward: the fp32-MFMA input-gradient kernel instead of the
                                           * split-bf16 one (the default where F_out % 32 == 0) */
#define PG_FLAG_NO_NGRAM (1u << 20)       /* host-side: use the CSR propagation kernels even if the graph has an n-gram plan */
#define PG_FLAG_NGRAM_BLOCK4 (1u << 21)   /* host-side: the 4x4-block n-gram forward (pg_spmm3_ngram_f32) instead of the
                                             middle-tile kernel (pg_spmm3_ngram_mid_f32) */
#define PG_FLAG_MID_NO_PAIRS (1u << 22)   /* middle-tile kernel: no workgroup pairs on odd / even feature chunks
                                             (each workgroup walks all chunks of its middles) */
#define PG_FLAG_MID_LOADER_SYNC (1u << 19) /* middle-tile kernels: the loader waits for chunk t+1's out / self rows
                                             before the in-phase barrier of chunk t (the round-3 protocol) instead of
                                             before the store-out barrier */
#define PG_FLAG_DENSE_NO_IL (1u << 13)    /* pipelined dense kernel: issue the next-but-one tile's A / gate LDS-DMA
                                             pieces all at the top of the iteration (the round-3 schedule) instead of
                                             between the MFMA k-steps (the default); same results */
#define PG_FLAG_DENSE_A_CACHED (1u << 12) /* pipelined dense kernels: default cache policy for the LDS-DMA of the
                                             A rows and the per-node constant instead of non-temporal (speed only) */
#define PG_FLAG_SCATTER_CPW_SHIFT 24    /* scatter kernel (pg_spmm3t_ngram_scatter_*): bits 24..28 = 16-feature chunks per
                                           workgroup (1..31, clamped to F / 16; 0 = chosen from the CU count) */
#define PG_FLAG_MID_TRANSPOSED (1u << 23) /* host-side: spmm3_t runs the transposed middle-tile kernels instead of the
                                             4x4-block ones: fp32 pg_spmm3t_ngram_mid_offdiag_f32 plus the diagonal
                                             term on the host, bf16 pg_spmm3t_ngram_mid_bf16 */

/* `row_order` (all SpMM entry points): optional int32 [n_rows] permutation giving the order in which
 * destination rows are processed (position p handles row row_order[p]; NULL = 0..n_rows-1). It changes
 * only the schedule -- which rows run concurrently on one XCD and share its L2 -- never the result.
 * The n-gram builder orders rows by (min out-neighbour, min in-neighbour), which groups the rows that
 * share their out-neighbour set (same (n-1)-suffix) and in-neighbour set (same (n-1)-prefix). */

const char* pg_last_error(void);
int pg_abi_version(void);

/* Z[i, 0:F] = sum_e w_in*X[col], Z[i, F:2F] = sum_e w_out*X[col], Z[i, 2F:3F] = sum_e w_und*X[col]
 * over row i of the shared pattern. One pass: each X row gathered once per pattern entry.
 * Replaces the 3 x 2 propagate calls of protgram_directgcn.py:101-112 (aggregate-then-transform).
 * Requirements: ldx >= F, ldz >= 3F, n_rows rows in rowptr (n_rows+1 entries), col < rows(X). */
int pg_spmm3_f32(int64_t n_rows, const int64_t* rowptr, const int32_t* row_order, const pg_edge3_t* edges,
                 const float* X, int64_t ldx, int64_t F,
                 float* Z, int64_t ldz, uint32_t flags, void* stream);


/* Same output as pg_spmm3_f32, with the three propagation weights computed in-kernel from raw counts
 * (graph_utils.py:198-273 closed form; bit-exact to the reference's torch.sparse construction) and
 * the per-node terms `node_norm` ([n_nodes, 4] as described above). eps = GCN_PROPAGATION_EPSILON. */
int pg_spmm3_fusednorm_f32(int64_t n_rows, const int64_t* rowptr, const int32_t* row_order,
                           const pg_edgeraw_t* edges,
                           const float* node_norm, float eps,
                           const float* X, int64_t ldx, int64_t F,
                           float* Z, int64_t ldz, uint32_t flags, void* stream);

/* Materialise the precomputed-weight records from raw records (same closed form as fused mode). */
int pg_edges_normalize_f32(int64_t n_rows, const int64_t* rowptr, const pg_edgeraw_t* raw,
                           const float* node_norm, float eps, pg_edge3_t* out, void* stream);

/* Transposed propagation (backward of pg_spmm3_f32): dX[j, :] = sum_k sum_{e in row j of A_k^T}
 * w_k * G[col, kF:(k+1)F]. `edges` is the CSR of the TRANSPOSED pattern (keyed by source), or the
 * forward CSR itself when all three matrices are symmetric (n-gram graphs: SURVEY §8a A10).
 * If accumulate != 0, dX += result. */
int pg_spmm3t_f32(int64_t n_rows, const int64_t* rowptr, const int32_t* row_order, const pg_edge3_t* edges,
                  const float* G, int64_t ldg, int64_t F,
                  float* dX, int64_t lddx, int accumulate, uint32_t flags, void* stream);

/* Single adjacency: Y[i, :] (+)= sum_e w * X[col, :]. Used for non-shared patterns (one call per
 * adjacency writing its column block of Z) and their transposes. */
int pg_spmm1_f32(int64_t n_rows, const int64_t* rowptr, const int32_t* row_order, const pg_edge1_t* edges,
                 const float* X, int64_t ldx, int64_t F,
                 float* Y, int64_t ldy, int accumulate, uint32_t flags, void* stream);

/* Dense DirectGCN contraction + combine on MFMA (v_mfma_f32_32x32x2_f32, exact fp32 products).
 * Given the three aggregates Z = [A_in X | A_out X | A_und X] ([M, 3*F_in]), computes per row m
 *   y[m] = s_in[m]  * (Z_in[m]  (W_main_in  + W_shared)^T + b_main_in  + b_dir_shared_in)
 *        + s_out[m] * (Z_out[m] (W_main_out + W_shared)^T + b_main_out + b_dir_shared_out)
 *        + s_und[m] * (Z_und[m] (W_undirected + W_shared)^T + b_undirected + b_undirected_shared)
 *        + constant[r(m)]                                    (vector-coefficient mode only)
 *   s_in = c_all*c_dir*c_in, s_out = c_all*c_dir*c_out, s_und = c_all*c_und,  c_x = C_x_vec[r(m)] or C_x[0]
 *   r(m) = rows ? rows[m] : m                                 (original_indices, :116-120)
 * which is protgram_directgcn.py:100-133 with A(xW) = (Ax)W. Optionally fused after it
 * (ProtGramDirectGCN.forward :213-215): + residual (res_x[m] when W_res == NULL, else
 * res_x[m] W_res^T + b_res as a 4th K segment), then leaky_relu(slope) when act != 0.
 * All weights are nn.Linear layout [F_out, F_in] with leading dimension F_in (contiguous). */
#define PG_GATES_VECTOR 0
#define PG_GATES_SCALAR 1

typedef struct pg_layer_args {
    int64_t M, F_in, F_out;
    const float* Z; int64_t ldz;
    const float* W_main_in; const float* W_main_out; const float* W_undirected; const float* W_shared;
    const float* b_main_in; const float* b_dir_shared_in;
    const float* b_main_out; const float* b_dir_shared_out;
    const float* b_undirected; const float* b_undirected_shared;
    int32_t gate_mode;
    const float* C_in; const float* C_out; const float* C_directed; const float* C_undirected; const float* C_all;
    const int64_t* rows;
    const float* constant; int64_t ld_const;
    const float* res_x; int64_t ld_res;
    const float* W_res; const float* b_res;
    int32_t act; float slope;
    float* Y; int64_t ldy;
    /* Fused layer dropout (the F.dropout after each layer, protgram_directgcn.py:216), applied after the activation
     * by the dense forward: output element m * F_out + j is kept when a counter-based hash of (*drop_seed, index)
     * passes p, and scaled by 1 / (1 - p). drop_p = 0: none. Needs act. The dense backward takes the same drop_p and
     * recovers the mask from the stored output Y (drop_seed is not read there). */
    float drop_p; const int64_t* drop_seed;
} pg_layer_args_t;

/* Number of floats of the packed operand: B = [W_mi+W_s | W_mo+W_s | W_u+W_s (| W_res)] as [F_out, K]
 * (K = 3*F_in, or 4*F_in with a projected residual) followed by the bias sums [4, F_out]
 * (b_main_k + b_shared_k for k = in, out, und; then b_res or 0). */
int64_t pg_directgcn_packed_floats(int64_t F_in, int64_t F_out, int has_res_proj);

/* Pack the weights/biases named in `args` (W_*, b_*, W_res, b_res) into `packed` (device memory of
 * pg_directgcn_packed_floats() floats). Re-run only when the parameters change. */
int pg_directgcn_pack_f32(const pg_layer_args_t* args, float* packed, void* stream);

/* The contraction + epilogue. Reads weights/biases from `packed` (the W_* / b_* fields of args are not
 * read); W_res != NULL selects the projected residual. packed == NULL: the kernel forms W_q + W_shared and the
 * bias sums from the W_* / b_* fields itself (the pack kernel's fp32 adds, so the result is identical), which
 * only the pipelined split-bf16 kernel does (F_in = F_out = 128, no W_res, no row map, 16-B aligned weights);
 * any other case returns PG_ERR_UNSUPPORTED without launching (callers then pack and call again). */
int pg_directgcn_dense_f32(const pg_layer_args_t* args, const float* packed, uint32_t flags, void* stream);

/* pg_directgcn_dense_f32 over the rows of a middle range in middle-major order (the rows
 * pg_spmm3_ngram_mid_rows_f32 writes: row m = 400 (M - m0) + 20 a + b for the middles m0, m0 + 1, ..., K = 20),
 * with the residual rows read (map_res != 0) and / or the output rows written (map_y != 0) at the global n-gram
 * row a.M.b = a Kn1 + 20 M + b (Kn1 = K^(n-1)) of res_x / Y instead of at row m: a rank of the multi-GPU middle
 * partition reads its layer input and writes its layer output in the global row layout directly (no row gather /
 * scatter around the launch). Same arithmetic as pg_directgcn_dense_f32 (bit-identical rows). Only the pipelined
 * split-bf16 kernel's shape (F_in = F_out = 128, no W_res, no rows, 16-B aligned): PG_ERR_UNSUPPORTED otherwise.
 * Requires K = 20 (Kn1 a power of 20), args->M a multiple of 400 and m0 + M / 400 <= Kn1 / 20. (Replaces, for a middle range, the same
 * protgram_directgcn.py:100-133 + :213-215 as pg_directgcn_dense_f32.) */
int pg_directgcn_dense_ngram_rows_f32(const pg_layer_args_t* args, const float* packed, int64_t Kn1, int64_t m0,
                                      int32_t map_res, int32_t map_y, uint32_t flags, void* stream);

/* pg_spmm3_f32 with the DirectGCN gates applied at the store: Z_q[i] = s_q(i) * (A_q X)[i], s_in = c_all*c_dir*c_in,
 * s_out = c_all*c_dir*c_out, s_und = c_all*c_und (protgram_directgcn.py:116-133), from the C_* / gate_mode fields
 * of `gates` (rows must be NULL). The inference producer for pg_directgcn_dense_f32 with
 * PG_FLAG_DENSE_PREGATED (whose operand is exactly s_q * Z_q); training keeps the ungated Z for the gate
 * gradients. */
int pg_spmm3_gated_f32(int64_t n_rows, const int64_t* rowptr, const int32_t* row_order, const pg_edge3_t* edges,
                       const float* X, int64_t ldx, int64_t F, const pg_layer_args_t* gates,
                       float* Z, int64_t ldz, uint32_t flags, void* stream);

/* N-gram tile propagation (pg_ngram_spmm.hip). For a shared-pattern graph over ALL K^n n-grams (node id = the
 * base-K number of the n-gram, as the builder's sorted-string ids are when every n-gram occurs: data_builder.py
 * :164-175), the rows of each middle (n-2)-gram form a K x K grid whose out- and in-neighbour parts are dense
 * K x K blocks; a 4 x 4 sub-block is worked by two waves (forward: 2 a-rows x 4 b-columns each) or one
 * (transposed), which reuse every source row they load for 2-4 rows from registers (16 source rows per output
 * row in the forward at K = 20, 11 in the transposed, against the CSR's ~41). Same aggregates as pg_spmm3_f32 /
 * pg_spmm3_gated_f32 / pg_spmm3t_f32 (protgram_directgcn.py:101-112) up to fp32 summation order (FMA, slot
 * order); X must be finite (missing transitions are zero weights).
 *   pg_ngram_plan_floats: plan size in floats for (K, n, n_rows = K^n), or -1 when the shape is not supported
 *     (K a multiple of 4, n >= 2).
 *   pg_ngram_plan_f32: scatters the CSR's weights into the plan (zeroed first); *bad (device int) receives the
 *     number of entries that fit no slot -- a nonzero count means the graph is not an n-gram graph over K^n
 *     ids and the plan must not be used.
 *   pg_spmm3_ngram_f32: Z = [A_in X | A_out X | A_und X]; gates != NULL applies the DirectGCN gates at the store
 *     (as pg_spmm3_gated_f32). K = 20 (the amino-acid alphabet), F = 64, 128 or 256 (two column halves);
 *     PG_ERR_UNSUPPORTED otherwise.
 *   pg_spmm3t_ngram_f32: dX (+)= sum_k A_k G[:, kF:(k+1)F] for the symmetric n-gram matrices (A_k^T = A_k).
 *     F = 64, 128 or 256.
 *   pg_spmm3t_ngram_bf16: the transposed kernel on bf16 rows (the model's bf16 mode; replaces pg_spmm3t_bf16 on
 *     such graphs): fp32 sums, rounded once to bf16. F = 64, 128 or 256. */
int64_t pg_ngram_plan_floats(int K, int n, int64_t n_rows);
int pg_ngram_plan_f32(int K, int n, int64_t n_rows, const int64_t* rowptr, const pg_edge3_t* edges, float* plan,
                      int64_t plan_floats, int* bad, void* stream);
int pg_spmm3_ngram_f32(int K, int n, int64_t n_rows, const float* plan, const float* X, int64_t ldx, int64_t F,
                       const pg_layer_args_t* gates, float* Z, int64_t ldz, uint32_t flags, void* stream);
int pg_spmm3t_ngram_f32(int K, int n, int64_t n_rows, const float* plan, const float* G, int64_t ldg, int64_t F,
                        float* dX, int64_t lddx, int accumulate, uint32_t flags, void* stream);
int pg_spmm3t_ngram_bf16(int K, int n, int64_t n_rows, const float* plan, const uint16_t* G, int64_t ldg, int64_t F,
                         uint16_t* dX, int64_t lddx, int accumulate, uint32_t flags, void* stream);
/* pg_spmm3t_ngram_add_bf16: dX = C + sum_k A_k G[:, kF:(k+1)F] (bf16 rows, the sum in fp32, rounded once): the
 * accumulate form of pg_spmm3t_ngram_bf16 with the addend C read from its own rows (C may equal dX), so the caller's
 * C survives -- the bf16 layer backward's dpre, which is both the identity residual's gradient and the per-node
 * constant's (protgram_directgcn.py:101-112, :213-215). */
int pg_spmm3t_ngram_add_bf16(int K, int n, int64_t n_rows, const float* plan, const uint16_t* G, int64_t ldg,
                             int64_t F, const uint16_t* C, int64_t ldc, uint16_t* dX, int64_t lddx, uint32_t flags,
                             void* stream);

/* N-gram MIDDLE-tile propagation on the fp32 matrix cores (pg_ngram_mid.hip; replaces, on graphs over all K^n
 * n-grams, the six propagate calls of protgram_directgcn.py:101-112, like pg_spmm3_ngram_f32, and is the default
 * forward there). The rows a.M.b of one middle (n-2)-gram M form a K x K grid; per 16-feature column chunk its K^2
 * out-sources M.b.c, K^2 in-sources c.a.M and K^2 self rows are staged in LDS by LDS-DMA (loader waves, one phase
 * ahead), and each adjacency becomes two dense (3K x K) x (K x 16) products per grid column / row on
 * v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation), the out-part handed to the in-part through LDS.
 * One persistent workgroup per CU walks a contiguous range of the (middle, chunk) stream; the weights of a middle
 * (the plan, in MFMA fragment order) stay in registers across its chunks. K = 20; F a multiple of 16; 16-B aligned
 * X, Z rows; PG_ERR_UNSUPPORTED otherwise (no launch). Numerics: the reference's w*x terms summed in another
 * order: within fp32 rounding of it, not bit-exact; zero weights for missing transitions add 0*x, so X must be
 * finite (PG_FLAG_NO_NGRAM selects the bit-exact CSR kernels).
 *   pg_ngram_mplan_floats: middle-plan size in floats for (K, n, n_rows = K^n), or -1 (K != 20, n < 2).
 *   pg_ngram_mplan_f32: scatters the CSR's weights into the middle plan (zeroed first); *bad as pg_ngram_plan_f32.
 *   pg_spmm3_ngram_mid_f32: Z = [A_in X | A_out X | A_und X]; gates must be NULL (PG_ERR_UNSUPPORTED otherwise:
 *     the dense kernel applies the gates). */
int64_t pg_ngram_mplan_floats(int K, int n, int64_t n_rows);
int pg_ngram_mplan_f32(int K, int n, int64_t n_rows, const int64_t* rowptr, const pg_edge3_t* edges, float* plan,
                       int64_t plan_floats, int* bad, void* stream);
int pg_spmm3_ngram_mid_f32(int K, int n, int64_t n_rows, const float* plan, const float* X, int64_t ldx, int64_t F,
                           const pg_layer_args_t* gates, float* Z, int64_t ldz, uint32_t flags, void* stream);
/* The same kernel over the middles [m_begin, m_end) only (a rank's share in the middle partition, shard.py), X in
 * the global row layout (only the rows those middles read must be valid: their out-sources M.b.c, in-sources c.a.M
 * and own rows), Z in MIDDLE-MAJOR order: row (M - m_begin) K^2 + a K + b holds node a.M.b. */
int pg_spmm3_ngram_mid_rows_f32(int K, int n, int64_t n_rows, const float* plan, const float* X, int64_t ldx, int64_t F,
                                int64_t m_begin, int64_t m_end, float* Z, int64_t ldz, uint32_t flags, void* stream);
/* bf16 mode (config 5): the same kernels on bf16 rows of X and Z (ldx, ldz in elements; X rows 16-B aligned, Z rows
 * 8-B aligned), the weights, products and sums fp32, each aggregate rounded once to bf16 (RNE) at the store -- the
 * bf16 model's contract (every sum fp32, one rounding), as pg_spmm3_bf16. Sources are staged as bf16 (half the LDS
 * and HBM bytes of the fp32 kernel) and widened exactly when read. */
int pg_spmm3_ngram_mid_bf16(int K, int n, int64_t n_rows, const float* plan, const uint16_t* X, int64_t ldx, int64_t F,
                            uint16_t* Z, int64_t ldz, uint32_t flags, void* stream);
int pg_spmm3_ngram_mid_rows_bf16(int K, int n, int64_t n_rows, const float* plan, const uint16_t* X, int64_t ldx,
                                 int64_t F, int64_t m_begin, int64_t m_end, uint16_t* Z, int64_t ldz, uint32_t flags,
                                 void* stream);
/* Builder-produced graphs (run_graph_builder.py -> data_builder.py:29-35, 164-173): node ids are the sorted-string
 * ranks of the n-grams PRESENT, over an alphabet that includes the padding ' ' (and rare letters), so N != 20^n and
 * the grid arithmetic of the kernels above does not hold for node ids. The MAPPED form runs the same middle-tile
 * kernel on the K = 20 grid of the standard letters with a row map:
 *   ginv [n_nodes] int32: grid row (base-20 n-gram) of node i, -1 when the n-gram has a non-standard character;
 *   gmap [K^n] int32:     node row of grid row g, -1 when that n-gram is not a node.
 * pg_ngram_mplan_map_f32: the middle plan of the grid part (zeroed first); resid[e] (uint8, one per CSR entry) = 1
 *   for every entry that does not go to a grid slot (an end off the grid, or no out / in / diagonal slot), else 0.
 * pg_spmm3_ngram_mid_map_f32: Z = the grid part of [A_in X | A_out X | A_und X] at the node rows (X read at node
 *   rows gmap[.]; rows of nodes off the grid are NOT written). Same requirements and numerics as
 *   pg_spmm3_ngram_mid_f32; grid K^n < 2^31.
 * pg_spmm3_resid_f32: the residual pass -- list position i (rows[i] = node row, bit 31 set = add to Z instead of
 *   overwriting) over the compact CSR entries [rowptr[i], rowptr[i + 1]) of pg_edge3_t records: Z[row] (+)= the three
 *   aggregates of those entries (fp32 sums in entry order, 16-B aligned X / Z rows, F % 4 == 0). */
int pg_ngram_mplan_map_f32(int K, int n, int64_t n_nodes, const int64_t* rowptr, const pg_edge3_t* edges,
                           const int32_t* ginv, float* plan, int64_t plan_floats, uint8_t* resid, void* stream);
int pg_spmm3_ngram_mid_map_f32(int K, int n, const float* plan, const int32_t* gmap, const float* X, int64_t ldx,
                               int64_t F, float* Z, int64_t ldz, uint32_t flags, void* stream);
int pg_spmm3_resid_f32(int64_t n_list, const int64_t* rowptr, const int32_t* rows, const pg_edge3_t* edges,
                       const float* X, int64_t ldx, int64_t F, float* Z, int64_t ldz, uint32_t flags, void* stream);
/* Transposed middle-tile kernel, off-diagonal part: dX (+)= sum_k (A_k - Diag_k) G[:, kF:(k+1)F] for the symmetric
 * n-gram matrices (A_k^T = A_k; the backward of the six propagates, protgram_directgcn.py:101-112, replacing
 * pg_spmm3t_ngram_f32 / pg_spmm3t_f32 on graphs over all K^n n-grams), where Diag_k holds the middle plan's diagonal
 * slots (a self-loop of a constant n-gram sits in its out-slot and IS included). The caller adds
 * sum_k Diag_k G_k: the dense backward while it holds G (pg_directgcn_dense_bwd_f32 with `diag`), or the host
 * (ops.spmm3_t under PG_FLAG_MID_TRANSPOSED). Same middle plan and chunk stream as the forward; accumulate: dX +=.
 * K = 20, F a multiple of 16, 16-B aligned G and dX rows, K^n * ldg and K^n * lddx < 2^32; PG_ERR_UNSUPPORTED
 * otherwise. Numerics: within fp32 rounding of the CSR kernel; G must be finite. */
int pg_spmm3t_ngram_mid_offdiag_f32(int K, int n, int64_t n_rows, const float* plan, const float* G, int64_t ldg,
                                    int64_t F, float* dX, int64_t lddx, int accumulate, uint32_t flags, void* stream);
/* bf16 transposed middle-tile kernel, the FULL product (diagonal included): dX (+)= sum_k A_k G[:, kF:(k+1)F] on bf16
 * G and dX rows (fp32 weights and sums, dX rounded once, RNE; the same product as pg_spmm3t_ngram_bf16 on graphs over
 * all K^n n-grams, which stays ops.spmm3_t's default: this kernel measured slower). The half-size rows leave
 * LDS room for each slice's own rows, so the diagonal term costs a third read of G but no caller work. Same shape /
 * alignment rules as the fp32 kernel (16-B aligned bf16 rows). */
int pg_spmm3t_ngram_mid_bf16(int K, int n, int64_t n_rows, const float* plan, const uint16_t* G, int64_t ldg, int64_t F,
                             uint16_t* dX, int64_t lddx, int accumulate, uint32_t flags, void* stream);

/* Transposed middle-tile propagation of ONE middle-partition rank (shard.MiddleTrainer's backward, replacing the
 * transposed CSR pass pg_spmm3t_f32 / pg_spmm3t_bf16 over the rank's column block): G = dZ [n_mid * 400, ldg] of
 * the rank's owned rows a.M.b (middles M = m0 .. m0 + n_mid - 1, middle-major, (a, b) inside, the order
 * pg_spmm3_ngram_mid_rows_* writes), T [3 * n_mid * 400, ldt] fp32 = the three parts of sum_k A_k^T G_k that the
 * owned middles send to their row sets, each row written once (no accumulation, deterministic):
 *   D: row          l*400 + a*20 + b  <- row a.M.b   sum_k Wdiag_k[a,b] G_k[a.M.b]
 *   P: n_own  +     l*400 + b*20 + c  <- row M.b.c   sum_{k,a} Wout_k[a,b,c] G_k[a.M.b]
 *   S: 2 n_own +    l*400 + c*20 + a  <- row c.a.M   sum_{k,b} Win_k[a,b,c] G_k[a.M.b]
 * (l = M - m0, n_own = n_mid * 400). The caller sums the parts of each global row (pg_rows_gather_sum). `splan` =
 * pg_ngram_scatter_plan of the same middles (78,000 floats per middle). F a multiple of 16; 16-B aligned G (ldg a
 * multiple of 8 bf16 / 4 fp32 elements) and T. Numerics: fp32 MFMA sums of the same w*g terms (bf16 G widened
 * exactly): within fp32 rounding of the CSR transposed kernel. */
int pg_ngram_scatter_plan(int K, int n, const float* mplan, int64_t m0, int64_t n_mid, float* splan, void* stream);
int pg_spmm3t_ngram_scatter_f32(const float* splan, int64_t n_mid, const float* G, int64_t ldg, int64_t F, float* T,
                                int64_t ldt, uint32_t flags, void* stream);
int pg_spmm3t_ngram_scatter_bf16(const float* splan, int64_t n_mid, const uint16_t* G, int64_t ldg, int64_t F,
                                 float* T, int64_t ldt, uint32_t flags, void* stream);

/* Row gather / scatter by an int64 index list (shard.py's ghost-row exchange; replaces the torch index gather /
 * index_copy_ around the RCCL all_to_all, which have no reference counterpart: the reference is single-device).
 * Byte-generic rows of row_bytes (a multiple of 4; 16-B pieces when rows, strides and pointers allow); strides in
 * bytes. pg_rows_gather: dst[i] = src[idx[i]]; pg_rows_scatter: dst[idx[i]] = src[i] (indices must be distinct). */
int pg_rows_gather(const void* src, int64_t ld_src, const int64_t* idx, int64_t n, int64_t row_bytes, void* dst,
                   int64_t ld_dst, void* stream);
int pg_rows_scatter(const void* src, int64_t ld_src, const int64_t* idx, int64_t n, int64_t row_bytes, void* dst,
                    int64_t ld_dst, void* stream);
/* out[i] = sum of the rows listed for i, in list order, in fp32: entry idx[e] >= 0 is row idx[e] of A (fp32,
 * stride lda elements), idx[e] < 0 row -1 - idx[e] of B (bf16 if b_bf16 else fp32, stride ldb); entries of row i
 * are rowptr[i] .. rowptr[i+1]-1; out [n_out, F] fp32, or bf16 (one rounding) if out_bf16. F a multiple of 4. (The
 * middle partition's backward: a row's scatter parts plus the rows received for it from the other ranks.) */
int pg_rows_gather_sum(const float* A, int64_t lda, const void* B, int64_t ldb, int b_bf16, const int64_t* rowptr,
                       const int32_t* idx, int64_t n_out, int64_t F, void* out, int64_t ldo, int out_bf16,
                       void* stream);

/* Backward of pg_directgcn_dense_f32 (the autograd of protgram_directgcn.py:100-133 and the fused
 * residual / leaky_relu of :213-215). `args` is the forward's argument block, with Y = the forward output
 * (read for leaky_relu' when act != 0); `packed` the forward's packed operand. Outputs:
 *   dpre  [M, F_out]  = dY * leaky'(Y)         (also the identity residual's and the constant's gradient)
 *   dZ    [M, 3F_in]  = s_q * (dpre B_q)        gradient of the propagated aggregates (NULL: not needed)
 *   dres  [M, F_in]   = dpre W_res              projected residual only (W_res != NULL)
 *   dgate [5, M]      per-row dL/d{c_in, c_out, c_directed, c_undirected, c_all} (row m uses gate row r(m))
 *   gates [M, 4]      the row gates s_in, s_out, s_und, 1 (scratch output)
 *   dW    [F_out*K + 4*F_out]  dL/dB in the packed layout: segment q of [F_out, K] is the gradient of
 *                     W_main_q + W_shared (W_res for q = 3); then [4, F_out] for the bias sums (b_res last)
 * work: pg_directgcn_dense_bwd_workspace(args) floats. Deterministic (fixed-order reductions).
 * Returns PG_ERR_UNSUPPORTED unless F_in, F_out and every leading dimension are multiples of 4 and the
 * buffers 16-B aligned. Five launches on `stream`: transpose, dgrad (MFMA), gate grads, wgrad (MFMA,
 * split over rows), split reduction. Where F_out % 32 == 0 dgrad runs on the bf16 matrix cores in the exact
 * three-way split (six bf16 products per fp32 product, fp32 sums; the transpose also splits the packed weights),
 * unless flags has PG_FLAG_DGRAD_F32MFMA (the fp32-MFMA kernel). */
typedef struct pg_layer_grad_args {
    const float* dY; int64_t lddy;
    float* dpre; int64_t ldp;
    float* dZ; int64_t lddz;
    float* dres; int64_t lddres;
    float* dgate;
    float* gates;
    float* dW;
    float* work; int64_t work_floats;
    /* optional (bf16 backward only; NULL: not written): dpre as fp32, the same bf16-rounded values -- the per-node
     * constant's gradient in its fp32 parameter dtype without a conversion pass */
    float* dpre_f32; int64_t ldp_f32;
} pg_layer_grad_args_t;

int64_t pg_directgcn_dense_bwd_workspace(const pg_layer_args_t* args);
int pg_directgcn_dense_bwd_f32(const pg_layer_args_t* args, const float* packed, const pg_layer_grad_args_t* grads,
                               uint32_t flags, void* stream);

/* pg_directgcn_dense_bwd_f32 that also writes the transposed propagation's diagonal term of the layer input's
 * gradient (the autograd of protgram_directgcn.py:101-112 for the rows' own entries; with e_res, plus the identity
 * residual's gradient dpre, :213-215):
 *   E[m, f] = sum_q wdiag[m, q] * dZ_q[m, f]  (+ dpre[m, f])          m < M, f < F_in, row stride lde
 * wdiag = the diagonal entries A_q[m, m] as fp32 [M, 3] (q = in, out, und; NgramPlan.diag3()). Each workgroup's
 * n-tile spans the three segments of 64 features, so the term comes from the accumulators (dgrad_span_kernel); the
 * caller then accumulates the off-diagonal part into E (pg_spmm3t_ngram_mid_offdiag_f32 with accumulate = 1), which
 * makes E the input's whole gradient. Same outputs as pg_directgcn_dense_bwd_f32 otherwise (dZ required). Needs
 * F_in % 64 == 0, F_out % 32 == 0, no projected residual (W_res == NULL), no row map (rows == NULL), F_in == F_out
 * when e_res, the vector path's alignment, E 16-B aligned and lde % 4 == 0 (else PG_ERR_UNSUPPORTED). */
int pg_directgcn_dense_bwd_span_f32(const pg_layer_args_t* args, const float* packed, const pg_layer_grad_args_t* grads,
                                    const float* wdiag, float* E, int64_t lde, int e_res, uint32_t flags, void* stream);

/* ---- bf16 mode (config 5: bf16 storage, fp32 accumulation) --------------------------------------
 * Features, aggregates, layer outputs and their gradients are bf16 (uint16_t bit patterns); every sum is
 * fp32, rounded once to bf16 (round-to-nearest-even, as torch) when stored. Parameters stay fp32. */

/* out[i] = bf16(in[i]) (e.g. the packed contraction operand of pg_directgcn_pack_f32). */
int pg_f32_to_bf16(int64_t n, const float* in, uint16_t* out, void* stream);

/* pg_spmm3_f32 over bf16 rows: Z = bf16([A_in X | A_out X | A_und X]), fp32 FMA sums in the same entry
 * order as pg_spmm3_f32 (so within one bf16 rounding of bf16(pg_spmm3_f32(X))). F in {16,32,64,128,256,512}; F, ldx, ldz multiples of 8; 16-B aligned (else
 * PG_ERR_UNSUPPORTED). */
int pg_spmm3_bf16(int64_t n_rows, const int64_t* rowptr, const int32_t* row_order, const pg_edge3_t* edges,
                  const uint16_t* X, int64_t ldx, int64_t F, uint16_t* Z, int64_t ldz, uint32_t flags, void* stream);

/* Transpose of pg_spmm3_bf16 (backward): dX[i] = bf16(sum_e w_in G[col,0:F] + w_out G[col,F:2F] + w_und G[col,2F:3F])
 * over the transposed CSR (= the forward CSR for symmetric matrices). */
int pg_spmm3t_bf16(int64_t n_rows, const int64_t* rowptr, const int32_t* row_order, const pg_edge3_t* edges,
                   const uint16_t* G, int64_t ldg, int64_t F, uint16_t* dX, int64_t lddx, uint32_t flags,
                   void* stream);

/* pg_directgcn_dense_f32 on bf16 MFMA (v_mfma_f32_32x32x16_bf16). In `args`, Z, res_x and Y point to bf16
 * data (their float* types are reinterpreted); gates, constant and the bias sums (read from the fp32
 * `packed`) stay fp32. `packed_bf16` = pg_f32_to_bf16 of the first F_out*K floats of `packed`. Needs
 * F_in % 8 == 0, F_out % 4 == 0, ldz and ld_res multiples of 8, 16-B aligned Z / res_x / packed_bf16 /
 * constant, 8-B aligned Y (else PG_ERR_UNSUPPORTED). */
int pg_directgcn_dense_bf16(const pg_layer_args_t* args, const float* packed, const uint16_t* packed_bf16,
                            uint32_t flags, void* stream);

/* pg_directgcn_dense_bwd_f32 in bf16 mode (bf16 MFMA products, fp32 sums): in `args` Z, res_x and Y are
 * bf16, in `grads` dY, dpre, dZ and dres are bf16; dgate, gates, dW and work stay fp32. Same workspace
 * (pg_directgcn_dense_bwd_workspace) and output layout as the fp32 entry point. Needs F_in, F_out and
 * every leading dimension a multiple of 8 and 16-B aligned buffers (else PG_ERR_UNSUPPORTED). */
int pg_directgcn_dense_bwd_bf16(const pg_layer_args_t* args, const float* packed, const uint16_t* packed_bf16,
                                const pg_layer_grad_args_t* grads, uint32_t flags, void* stream);

/* pg_directgcn_head_f32 with a bf16 input h (bf16 mode); outputs stay fp32. Needs the fast-path shape
 * (F <= 256, H <= 128, C <= 64; F, H, ldh, lde multiples of 4), else PG_ERR_UNSUPPORTED. */
int pg_directgcn_head_bf16(int64_t M, int64_t F, int64_t H, int64_t C, const uint16_t* h, int64_t ldh,
                           const float* W1, const float* b1, const float* W2, const float* b2, float eps,
                           float* logp, int64_t ldp, float* emb, int64_t lde, void* stream);

/* n-gram transition producer (data_builder.py:38-54 windows as integer keys). For sequence s, positions
 * p in [offsets[s], offsets[s+1]) of `bytes`: keys[p] = sum_j lut[bytes[p+j]] * K^(n-1-j) for the window
 * [p, p+n) if it lies inside the sequence, else -1; next_keys[p] = key of window p+1 if the transition
 * p -> p+1 (window [p+1, p+n+1)) lies inside the sequence, else -1. `lut` [256] maps a byte to its
 * order-preserving code in [0, K). K^n must fit 63 bits (PG_ERR_ARG otherwise). */
int pg_ngram_keys(int64_t nseq, const int64_t* offsets, const uint8_t* bytes, const int32_t* lut, int n,
                  int64_t K, int64_t* keys, int64_t* next_keys, void* stream);

/* ---- training-step helpers (the trainer's L2 term over all parameters, trainer :96 / :136) ---------
 * A tensor list is a device array of descriptors; tensor t is split into pg_multi_chunks(numel_t) chunks of
 * 16K elements and chunk_ptr[t] = the first chunk of tensor t (exclusive prefix sum, chunk_ptr[ntens] =
 * nchunks). */
typedef struct pg_tensor_desc {
    const float* x;  /* read */
    float* y;        /* written by pg_multi_axpy_f32 (unused by pg_multi_sqsum_f32) */
    int64_t numel;
} pg_tensor_desc_t;

int64_t pg_multi_chunks(int64_t numel);

/* out[0] = sum_t sum_i x_t[i]^2, fixed-order reduction (deterministic). partial: nchunks floats. */
int pg_multi_sqsum_f32(int ntens, const pg_tensor_desc_t* descs, const int64_t* chunk_ptr, int64_t nchunks,
                       float* partial, float* out, void* stream);

/* y_t[i] += a * x_t[i] for every tensor of the list (one launch), a = alpha * (alpha_scale ? *alpha_scale : 1):
 * alpha_scale is a device scalar (e.g. GradScaler's scale, read without a host sync). */
int pg_multi_axpy_f32(int ntens, const pg_tensor_desc_t* descs, const int64_t* chunk_ptr, int64_t nchunks,
                      float alpha, const float* alpha_scale, void* stream);

/* Adam over a parameter list in one launch (torch.optim.Adam's update, amsgrad = maximize = False, L2-style
 * weight_decay): p, m (exp_avg), v (exp_avg_sq) updated in place from g; bias corrections from the device
 * step counter `step` (incremented afterwards unless *found_inf != 0). grad_scale / found_inf: GradScaler's
 * device scale (gradients are multiplied by 1/scale) and inf flag (update skipped), or NULL. */
typedef struct pg_adam_desc {
    float* p;
    const void* g;  /* fp32, or bf16 (uint16 bits) when gtype == 1 */
    float* m;
    float* v;
    int64_t numel;
    int64_t gtype;  /* 0: fp32 gradient; 1: bf16 gradient, widened exactly (ABI 4) */
} pg_adam_desc_t;

/* sq_partial (optional, [nchunks]): per-chunk sums of p^2 of the parameters BEFORE the update -- the value of the
 * trainer's L2 term (protgram_directgcn_trainer.py:96) from the pass that reads p anyway; written on skipped
 * (found_inf) steps too. pg_multi_sum_f32 adds n partials in fixed order (deterministic).
 * hyper (optional): device double[2] = {lr, weight_decay}. When given, the kernel reads the learning rate and the
 * decay there at run time (lr argument ignored; decay = hyper[1] + weight_decay argument), so a step captured in a
 * HIP graph follows the schedule the caller writes into it between replays (ReduceLROnPlateau,
 * protgram_directgcn_trainer.py:84, :102). Same arithmetic as the by-value form: the same bits. */
int pg_adam_f32(int ntens, const pg_adam_desc_t* descs, const int64_t* chunk_ptr, int64_t nchunks, double lr,
                double beta1, double beta2, double eps, double weight_decay, float* step, const float* grad_scale,
                const float* found_inf, float* sq_partial, const double* hyper, void* stream);
int pg_multi_sum_f32(int64_t n, const float* x, float* out, void* stream);

/* Training step of the prediction head (decoder_fc -> log_softmax -> nll_loss, protgram_directgcn.py:218-222 and
 * protgram_directgcn_trainer.py:91-100), forward and backward in one pass over the M rows of h [M, F]:
 *   a = dropout(relu(h W1^T + b1)), logits = a W2^T + b2, loss = loss_weight * sum_m -log_softmax(logits[m])[y[m]];
 * with s = *grad_scale (or 1): dh [M, F] and grads = [dW1 (H x F) | db1 (H) | dW2 (C x H) | db2 (C)] of s * loss;
 * loss[0] = the unscaled loss. drop_p > 0: keep element (m, j) of a by a counter-based draw from seed[0] (device
 * int64), scaled by 1 / (1 - drop_p). W1 [H, F], W2 [C, H] row-major (nn.Linear weights); y int64 [M].
 * F = 128, H = 64, C <= 32 only (PG_ERR_UNSUPPORTED otherwise). work: pg_head_train_workspace floats. */
int64_t pg_head_train_workspace(int64_t M, int64_t F, int64_t H, int64_t C);
int pg_head_train_f32(int64_t M, int64_t F, int64_t H, int64_t C, const float* h, int64_t ldh, const float* W1,
                      const float* b1, const float* W2, const float* b2, const int64_t* y, float loss_weight,
                      float drop_p, const int64_t* seed, const float* grad_scale, float* dh, int64_t lddh,
                      float* grads, float* loss, float* work, int64_t work_floats, void* stream);

/* The same step in the model's bf16 mode at F = 256, H = 128, C <= 32 (config 5's head): h and dh are bf16 rows (dh
 * rounded once); the products run on the bf16 matrix cores with two-term bf16 splits of the fp32 operands (each
 * product within ~2^-15 relative of fp32), fp32 sums; loss and grads fp32 as pg_head_train_f32. work:
 * pg_head_train_bf16_workspace floats; other shapes: PG_ERR_UNSUPPORTED (-1 from the workspace query). */
int64_t pg_head_train_bf16_workspace(int64_t M, int64_t F, int64_t H, int64_t C);
int pg_head_train_bf16(int64_t M, int64_t F, int64_t H, int64_t C, const uint16_t* h, int64_t ldh, const float* W1,
                       const float* b1, const float* W2, const float* b2, const int64_t* y, float loss_weight,
                       float drop_p, const int64_t* seed, const float* grad_scale, uint16_t* dh, int64_t lddh,
                       float* grads, float* loss, float* work, int64_t work_floats, void* stream);

/* Weight gradient of a row-wise linear map over many rows: out[0 : P*N] = A^T B ([P, N], row-major,
 * the sum running over the M rows of A [M, P] and B [M, N]) and out[P*N : P*N+P] = column sums of A.
 * For y = x W^T + b with A = dy, B = x this is (dW, db) of nn.Linear; the decoder layers of
 * protgram_directgcn.py:173-177 (M = graph nodes, P, N <= a few hundred) in training. Deterministic
 * split-K MFMA (same kernel as the dense backward). Needs P, N, lda, ldb multiples of 4 and 16-B aligned
 * buffers (else PG_ERR_UNSUPPORTED). work: pg_gemm_at_b_workspace(M, P, N) floats. */
int64_t pg_gemm_at_b_workspace(int64_t M, int64_t P, int64_t N);
int pg_gemm_at_b_f32(int64_t M, int64_t P, int64_t N, const float* A, int64_t lda, const float* B, int64_t ldb,
                     float* out, float* work, int64_t work_floats, void* stream);

/* The dense backward's weight and bias gradients laid out as the layer's parameters take them (the autograd of
 * protgram_directgcn.py:100-133 in nn.Linear / bias shapes), one launch instead of a transpose copy, two adds and a
 * bias copy: from dB [F_out, S * F_in] and dbsum [>= 3, F_out] (pg_directgcn_dense_bwd_*'s dW) writes
 * out = [S][F_out][F_in] (the gradients of W_main_in, W_main_out, W_undirected (, W_res): segment q of each row),
 * then [F_out][F_in] = (seg0 + seg1) + seg2 (W_shared: fp32 adds in that order), then [2][3][F_out] (b_main_q and
 * b_*_shared_q both receive dbsum[q]). out: (S + 1) F_out F_in + 6 F_out floats; S = 3 or 4. Needs F_in % 4 == 0
 * and 16-B aligned dB, out (else PG_ERR_UNSUPPORTED). */
int pg_dense_grads_layout_f32(int64_t F_out, int64_t F_in, int32_t S, const float* dB, const float* dbsum, float* out,
                              void* stream);

/* Fused prediction head (protgram_directgcn.py:218-222, eval mode): per row m of h [M, F]
 *   logp[m] = log_softmax(W2 relu(W1 h[m] + b1) + b2)      W1 [H, F], W2 [C, H] (nn.Linear layout)
 *   emb[m]  = h[m] / (||h[m]||_2 + eps)                      (models_utils.py:139-147)
 * One read of h; both products on fp32 MFMA for F <= 256, H <= 128, C <= 64, else a VALU kernel. */
int pg_directgcn_head_f32(int64_t M, int64_t F, int64_t H, int64_t C, const float* h, int64_t ldh,
                          const float* W1, const float* b1, const float* W2, const float* b2, float eps,
                          float* logp, int64_t ldp, float* emb, int64_t lde, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* PG_DIRECTGCN_H */
