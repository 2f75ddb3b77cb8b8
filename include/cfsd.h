/*
 * cfsd.h — C ABI of libcfsd.so, the MI355X (gfx950) kernels of the
 * spiral-convolution mesh-VAE training step (CraniofacialSD-VAE).
 *
 * The reference has no FFI: its hot path is the Python module API of
 * model.py / swap_batch_transform.py / model_manager.py running on ATen and
 * torch-scatter.  Each entry point below names the reference interface whose
 * arithmetic it replaces (path:line in simofoti/CraniofacialSD-VAE).
 *
 * Conventions (all entry points):
 *  - every pointer is a DEVICE pointer owned by the caller; the library never
 *    allocates device memory (workspaces are passed in);
 *  - tensors are dense row-major fp32, activations [batch, vertices, channels];
 *    index tables are int32;
 *  - launches are asynchronous on `stream` (a hipStream_t, may be NULL for the
 *    default stream) with no host synchronisation, so calls can be captured
 *    into a hipGraph;
 *  - the return value is CFSD_OK (0), a negative CFSD_E* code for invalid
 *    arguments, or a positive hipError_t; cfsd_last_error_string() gives text
 *    (per calling thread).  Nothing aborts and no C++ exception crosses the ABI.
 *  - stateless and re-entrant.
 */
#ifndef CFSD_H
#define CFSD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CFSD_OK 0
#define CFSD_EINVAL (-1)      /* bad shape / null pointer / unsupported size */
#define CFSD_EWORKSPACE (-2)  /* workspace too small */

#define CFSD_ACT_NONE 0
#define CFSD_ACT_ELU 1

/* Storage type of an activation / gradient operand of the mixed-precision
 * (bf16) entry points: fp32, or bfloat16 as raw uint16 (torch.bfloat16 bits). */
#define CFSD_DT_F32 0
#define CFSD_DT_BF16 1
/* Storage flag OR-ed into a *_dt argument of the mixed-precision entry points
 * (ABI 4.0): the operand is VERTEX-MAJOR.  A logical [batch, nv, c] tensor
 * then has element (b, v, k) at ((size_t)v * batch + b) * c + k, so the rows
 * of one vertex in every mesh of the batch are one contiguous block (torch:
 * an empty [nv, batch, c] tensor viewed through .permute(1, 0, 2)).  Without
 * the flag: batch-major, (b * nv + v) * c + k (the reference's [B, V, C]).
 * Each operand's layout is independent (e.g. E1 reads a vertex-major level-1
 * tensor and writes a batch-major level-2 one); results do not depend on the
 * layout.  Where one descriptor covers several operands, the entry point says
 * so. */
#define CFSD_VM 0x10
#define CFSD_DT_TYPE(dt) ((dt) & 0xf)

/* ABI version: (major << 16) | minor. */
int cfsd_version(void);
const char* cfsd_last_error_string(void);

/* ---------------------------------------------------------------- SpiralConv
 * Replaces SpiralConv.forward (model.py:27-41) + F.elu (model.py:68,84):
 *   y[b,r,o] = act( bias[o] + sum_{s,c} w[o, s*cin + c] * x[b, idx[r*seq+s], c] )
 * x [batch, vsrc, cin], idx [rows, seq] (values in [0, vsrc)), w [cout, seq*cin],
 * y [batch, rows, cout].  `rows` may be a subset of the mesh's vertices (the
 * Enblock evaluates the conv only where the 0/1 down-sample selects, which is
 * bit-identical to conv -> Pool(down) for a selection transform). */
int cfsd_spiral_conv_fwd(const float* x, const int32_t* idx, const float* w, const float* bias,
                         float* y, float* workspace, size_t workspace_bytes, int batch, int vsrc,
                         int rows, int seq, int cin, int cout, int act, void* stream);

/* Workspace (bytes) that lets cfsd_spiral_conv_fwd / _bwd_data split the
 * spiral slots of layers with few rows over more workgroups (partial sums
 * combined in a fixed order).  NULL/0 workspace is allowed for 32-channel
 * layers (no split); 64x64 layers require it. */
size_t cfsd_spiral_conv_workspace(int batch, int vsrc, int rows, int seq, int cin, int cout);

/* Replaces the autograd of model.py:34 (IndexSelectBackward = index_add_) and
 * :40 (AddmmBackward dX = dY.W), deterministically (no atomics):
 *   dx[b,u,c] = g(b,u,c) * sum_{(r,s): idx[r,s]=u} sum_o dpre[b,r,o] w[o, s*cin+c]
 * where g = elu'(elu_y[b,u,c]) computed from the ELU output when elu_y != NULL
 * (fuses the previous layer's ELU backward), else 1.
 * inv_ptr [vsrc*seq + 1] / inv_row [rows*seq]: CSR of the inverse spiral,
 * entry list of (u, s) = rows r with idx[r*seq+s] == u (r ascending);
 * inv_head [vsrc*seq][CFSD_INV_HEAD]: the first four entries of each list (-1
 * if absent, 16-B aligned rows), read up front with one load per key so the
 * gathers are issued without walking the CSR (required; inv_ptr/inv_row are
 * only read for lists longer than the head).  The spiral length must be 9
 * (all reference configs). */
#define CFSD_INV_HEAD 4
int cfsd_spiral_conv_bwd_data(const float* dpre, const int32_t* inv_ptr, const int32_t* inv_row,
                              const int32_t* inv_head, const float* w, const float* elu_y,
                              float* dx, float* workspace, size_t workspace_bytes, int batch,
                              int vsrc, int rows, int seq, int cin, int cout, void* stream);

/* Replaces AddmmBackward's dW = G^T.dY and db = sum dY (model.py:40):
 *   dw[o, s*cin+c] = sum_{b,r} dpre[b,r,o] x[b, idx[r,s], c],  db[o] = sum_{b,r} dpre[b,r,o]
 * Deterministic two-stage reduction through `workspace`
 * (cfsd_spiral_conv_bwd_weight_workspace() bytes). */
int cfsd_spiral_conv_bwd_weight(const float* x, const int32_t* idx, const float* dpre, float* dw,
                                float* db, float* workspace, size_t workspace_bytes, int batch,
                                int vsrc, int rows, int seq, int cin, int cout, void* stream);
size_t cfsd_spiral_conv_bwd_weight_workspace(int batch, int rows, int seq, int cin, int cout);

/* Deferred weight gradients.  cfsd_spiral_conv_bwd_weight / cfsd_spiral_conv_bwd
 * called with dw == db == NULL leave their per-workgroup partial sums in
 * `workspace` and skip the reduction; cfsd_dw_reduce_batch then reduces up
 * to 16 such layers (each with its own workspace) in ONE launch, with the
 * same fixed summation order (identical results).  `fused` = 1: the partials
 * came from cfsd_spiral_conv_bwd(_x) on a small-output layer (cout*seq <= 32);
 * 2: from cfsd_spiral_conv_bwd_weight_x on a 32/64-channel layer (bf16); 3: from
 * cfsd_spiral_conv_bwd_weight_x on a 32 -> 32 fp32 layer with vertex-major x
 * and dpre, batch % 16 == 0 (ABI 4.3), or from cfsd_spiral_conv_bwd_flat_pair
 * (ABI 4.10). */
typedef struct {
  const float* workspace;
  float* dw;
  float* db;
  int batch, vsrc, rows, cin, cout, fused;
} cfsd_dw_slabs;
int cfsd_dw_reduce_batch(const cfsd_dw_slabs* items, int n, void* stream);
/* cfsd_dw_reduce_batch fused with the Adam step of cfsd_adam (single-process
 * training, model_manager.py:316 after :315's backward): every item's dw/db
 * must lie inside the flat gradient `grad` [n_params]; each reduced element
 * is written to grad and updated in param / exp_avg / exp_avg_sq (and
 * param_bf16) by the thread that reduced it, every other element of the flat
 * buffers by extra workgroups of the same launch.  Same values as
 * cfsd_dw_reduce_batch followed by cfsd_adam. */
int cfsd_dw_reduce_batch_adam(const cfsd_dw_slabs* items, int n, float* param, const float* grad,
                              float* exp_avg, float* exp_avg_sq, const int32_t* step,
                              size_t n_params, float lr, float beta1, float beta2, float eps,
                              float weight_decay, uint16_t* param_bf16, void* stream);

/* Fused backward of one SpiralConv (model.py:27-41 autograd, dX and dW/db of
 * the same layer in one call): dx exactly as cfsd_spiral_conv_bwd_data
 * (skipped when dx == NULL, e.g. the first layer), dw/db exactly as
 * cfsd_spiral_conv_bwd_weight.  For small-output layers (cout*seq <= 32, the
 * xyz output conv) both come from ONE pass in source-row space: the spiral
 * transpose is folded in the 3-wide dpre space and dW is regrouped as
 * sum_{b,u} x[b,u,:] (x) t[b,u,s,:], so x is read densely, not gathered.
 * For coarse layers where cfsd_spiral_conv_bwd_paired() is 1, dx and the dW
 * slabs come from ONE launch whose workgroups interleave the two (same
 * results as the separate calls).
 * workspace: cfsd_spiral_conv_bwd_workspace() bytes (shared by both stages). */
int cfsd_spiral_conv_bwd(const float* x, const int32_t* idx, const float* dpre,
                         const int32_t* inv_ptr, const int32_t* inv_row, const int32_t* inv_head,
                         const float* w, const float* elu_y, float* dx, float* dw, float* db,
                         float* workspace, size_t workspace_bytes, int batch, int vsrc, int rows,
                         int seq, int cin, int cout, void* stream);
size_t cfsd_spiral_conv_bwd_workspace(int batch, int vsrc, int rows, int seq, int cin, int cout);
/* 1 when cfsd_spiral_conv_bwd with dx != NULL runs dx and dW as one paired
 * launch for this shape (no reference counterpart: a scheduling query). */
int cfsd_spiral_conv_bwd_paired(int batch, int vsrc, int rows, int seq, int cin, int cout);

/* Backward (dx and dW/db) of a conv evaluated on a ROW SUBSET (the Enblock
 * convs: `rows` = the kept vertices), in the reference's own two steps
 * (autograd of model.py:40 then :34): dG = dpre.W at the kept rows only
 * (MFMA, in the workspace), then dx[b,u,:] = g(b,u,:) * sum_{p in flat(u)}
 * dG[b, p, :] with flat(u) = the flattened spiral positions p = r*seq + s
 * having idx[r,s] == u, in ascending p (the sequential index_add_ order).
 * inv_flat [vsrc][flat_width] int32, -1 padded, 16-B aligned rows,
 * flat_width in {4, 8, 12, 16} (>= the largest fan-in).  dw/db exactly as
 * cfsd_spiral_conv_bwd_weight (dw == db == NULL defers: cfsd_dw_reduce_batch
 * item with fused = 1).  cin = 32, cout in {32, 64}.
 * workspace: cfsd_spiral_conv_bwd_rowsub_workspace() bytes (0 = unsupported). */
size_t cfsd_spiral_conv_bwd_rowsub_workspace(int batch, int vsrc, int rows, int seq, int cin,
                                             int cout);
int cfsd_spiral_conv_bwd_rowsub(const float* x, const int32_t* idx, const float* dpre,
                                const int32_t* inv_flat, int flat_width, const float* w,
                                const float* elu_y, float* dx, float* dw, float* db,
                                float* workspace, size_t workspace_bytes, int batch, int vsrc,
                                int rows, int seq, int cin, int cout, void* stream);
/* The feature swap (cfsd_swap_features_x: x = the swapped batch of bs^2
 * meshes from the resident set `data` [n_meshes][vsrc][3], in x_dt's layout)
 * and the first Enblock's xyz conv (cfsd_spiral_conv_fwd_x with cin = 3:
 * y = act(conv(x)) at the `rows` rows of idx) in ONE launch (ABI 4.9): the
 * conv gathers its inputs through the swap straight from `data`, so the two
 * are independent roles of the launch.  Same values as the two launches.
 * x fp32; y fp32 or bf16; cout 32 or 64. */
int cfsd_spiral_conv_fwd_in_swap(const float* data, const int32_t* batch_idx, const uint8_t* region_mask,
                                 const int32_t* key, int bs, int n_meshes, int n_regions, float* x, int x_dt,
                                 const int32_t* idx, const float* w, const float* bias, void* y, int y_dt,
                                 int vsrc, int rows, int cin, int cout, int act, void* stream);
/* Both gradients of a full 32 -> 32 SpiralConv (a Deblock conv, model.py:27-41
 * autograd) with EVERY operand vertex-major fp32 (x, dpre, dx, elu_y:
 * [vertex][batch][32]), batch % 16 == 0, batch x rows >= 65536, in ONE
 * launch (ABI 4.10): the flat-list data gradient of
 * cfsd_spiral_conv_bwd_data_flat (dx = elu'(elu_y) times the sum over u's
 * flat inverse list, elu_y may be NULL) and the weight-gradient slabs of
 * cfsd_spiral_conv_bwd_weight_x as interleaved workgroups, two per CU.
 * Bit-identical to those two calls.  dw == db == NULL defers
 * (cfsd_dw_reduce_batch item with fused = 3).  inv_flat as
 * cfsd_spiral_conv_bwd_data_flat (flat_width in {8, 12, 16, 20}).
 * workspace: cfsd_spiral_conv_bwd_flat_pair_workspace() bytes (0 = unsupported). */
size_t cfsd_spiral_conv_bwd_flat_pair_workspace(int batch, int rows, int seq, int cin, int cout);
int cfsd_spiral_conv_bwd_flat_pair(const float* x, const int32_t* idx, const float* dpre, const int32_t* inv_flat,
                                   int flat_width, const float* w, const float* elu_y, float* dx, float* dw,
                                   float* db, float* workspace, size_t workspace_bytes, int batch, int vsrc,
                                   int rows, int seq, int cin, int cout, void* stream);
/* The bf16 step's Enblock backward (ABI 4.11): the flat-list dx of
 * cfsd_spiral_conv_bwd_data_rowsub (fp32 batch-major dpre at the kept rows,
 * fp32 w, fp32 products; dx / elu_y bf16 vertex-major, rounded once) and the
 * weight-gradient slabs of cfsd_spiral_conv_bwd_weight_x (x bf16
 * vertex-major) as two workgroup roles of ONE launch; always deferred
 * (cfsd_dw_reduce_batch item with fused = 2).  32 -> 32, batch % 16 == 0,
 * flat_width in {4, 8, 12, 16}.  Same values as the two calls. */
int cfsd_spiral_conv_bwd_rowsub_pair_bf16(const void* x, const int32_t* idx, const float* dpre,
                                          const int32_t* inv_flat, int flat_width, const float* w, const void* elu_y,
                                          void* dx, float* workspace, size_t workspace_bytes, int batch, int vsrc,
                                          int rows, int seq, int cin, int cout, void* stream);
/* The same pair on the bf16 step's tensors (ABI 4.11): x, dpre, dx, elu_y
 * bf16 vertex-major, w the bf16 weight shadow; always deferred
 * (cfsd_dw_reduce_batch item with fused = 2; workspace as
 * cfsd_spiral_conv_bwd_weight_x_workspace).  Same values as
 * cfsd_spiral_conv_bwd_data_flat + cfsd_spiral_conv_bwd_weight_x. */
int cfsd_spiral_conv_bwd_flat_pair_bf16(const void* x, const int32_t* idx, const void* dpre, const int32_t* inv_flat,
                                        int flat_width, const void* w, const void* elu_y, void* dx, float* workspace,
                                        size_t workspace_bytes, int batch, int vsrc, int rows, int seq, int cin,
                                        int cout, void* stream);

/* The same with the source level's layout (ABI 4.4): x_dt = CFSD_DT_F32
 * [| CFSD_VM] describes x, dx and elu_y (the fp32 step's E1 reads and writes
 * the vertex-major level-1 tensors); dpre stays batch-major fp32.  Few-row
 * layers only (the dW slabs of conv_dw_lat). */
int cfsd_spiral_conv_bwd_rowsub_x(const float* x, int x_dt, const int32_t* idx, const float* dpre,
                                  const int32_t* inv_flat, int flat_width, const float* w, const float* elu_y,
                                  float* dx, float* dw, float* db, float* workspace, size_t workspace_bytes,
                                  int batch, int vsrc, int rows, int seq, int cin, int cout, void* stream);

/* dx alone of the row-subset backward (as cfsd_spiral_conv_bwd_rowsub):
 * dG = dpre.W (fp32 dpre and W, fp32 MFMA) in `workspace`
 * (cfsd_spiral_conv_bwd_data_rowsub_workspace() bytes), then the ascending
 * flat-list gather-sum with elu'(elu_y); dx and elu_y stored as dx_dt
 * (CFSD_DT_F32 or CFSD_DT_BF16: one rounding of the fp32 sum).  Used by the
 * bf16 path, whose dW comes from cfsd_spiral_conv_bwd_weight_x. */
size_t cfsd_spiral_conv_bwd_data_rowsub_workspace(int batch, int rows, int seq, int cin);
int cfsd_spiral_conv_bwd_data_rowsub(const float* dpre, const int32_t* inv_flat, int flat_width,
                                     const float* w, const void* elu_y, void* dx, int dx_dt,
                                     float* workspace, size_t workspace_bytes, int batch, int vsrc,
                                     int rows, int seq, int cin, int cout, void* stream);

/* Materialising spiral gather, g[b,r,s*cin+c] = x[b, idx[r,s], c]
 * (model.py:34 index_select + view).  Used as the HBM-roofline probe. */
int cfsd_spiral_gather(const float* x, const int32_t* idx, float* g, int batch, int vsrc, int rows,
                       int seq, int cin, void* stream);

/* ---------------------------------------------------------------- Pool
 * Replaces Pool (model.py:50-55: index_select * value, torch_scatter.scatter_add)
 * and its autograd, as a row-sorted CSR SpMM whose per-row order is the COO
 * file order (so the fp32 sum order equals the reference's sequential
 * scatter_add):
 *   y[b,r,:] = g(b,r,:) * sum_{k in row r} val[k] * x[b, col[k], :]
 * with g = elu'(elu_y) when elu_y != NULL (fuses the ELU backward of the
 * tensor the transpose product returns a gradient for), else 1.
 * x [batch, n, c], y [batch, m, c]; c % 4 == 0. */
int cfsd_spmm_csr(const int32_t* row_ptr, const int32_t* col, const float* val, const float* x,
                  const float* elu_y, float* y, int batch, int m, int n, int c, void* stream);

/* cfsd_spmm_csr(_x) for matrices with long, skewed rows (the up-sampling
 * transposes): same results bit for bit; rows are visited in `order` (a
 * permutation of [0, m), rows by decreasing length: the longest sequential
 * folds start first) and each row's entry list is prefetched one chunk ahead.
 * x / elu_y / y storage types as cfsd_spmm_csr_x. */
int cfsd_spmm_csr_sched(const int32_t* row_ptr, const int32_t* col, const float* val,
                        const int32_t* order, const void* x, int x_dt, const void* elu_y, void* y,
                        int y_dt, int batch, int m, int n, int c, void* stream);

/* cfsd_spmm_csr_sched with the CSR stored in visiting order: slot i (0..m-1)
 * is output row rows_s[i] (a permutation of [0, m)) with entries
 * [ptr_s[i], ptr_s[i+1]) of col_s / val_s, each row's entries in the original
 * per-row (file) order (topology.scheduled_csr).  Same results bit for bit as
 * cfsd_spmm_csr_x; one dependent index load fewer than cfsd_spmm_csr_sched. */
int cfsd_spmm_sched_csr(const int32_t* ptr_s, const int32_t* col_s, const float* val_s,
                        const int32_t* rows_s, const void* x, int x_dt, const void* elu_y, void* y,
                        int y_dt, int batch, int m, int n, int c, void* stream);

/* cfsd_spmm_csr_x for a matrix whose rows all hold exactly k (1..4) entries,
 * row r's at [r*k, r*k + k) of col/val (the CSR arrays of the barycentric
 * up-sampling matrices, Pool(up) at model.py:84 via model.py:50-55: 3 per
 * row).  No row_ptr: one dependent load fewer per row.  Same results bit for
 * bit as cfsd_spmm_csr_x on the same CSR. */
int cfsd_spmm_uniform(int k, const int32_t* col, const float* val, const void* x, int x_dt,
                      const void* elu_y, void* y, int y_dt, int batch, int m, int n, int c,
                      void* stream);

/* ---------------------------------------------------------------- feature swap
 * Replaces SwapFeatures.__call__ / swap (swap_batch_transform.py:13-52):
 *   out[i*bs+j, v, :] = x[mesh[(i != j && mask[key*nv + v]) ? j : i], v, :]
 * x [n_meshes, nv, c] resident dataset, batch_idx [bs] device indices of the
 * base meshes, region_mask [n_regions, nv] (1 = feature vertex of the region),
 * key: device int32 scalar (region index).  Bit-exact copy.  Device values
 * are range-guarded (never fault): a key outside [0, n_regions) swaps nothing,
 * a mesh index outside [0, n_meshes) is clamped. */
int cfsd_swap_features(const float* x, const int32_t* batch_idx, const uint8_t* region_mask,
                       const int32_t* key, float* out, int bs, int nv, int c, int n_meshes,
                       int n_regions, void* stream);
/* The same with the output's layout: out_dt = CFSD_DT_F32 [| CFSD_VM] (ABI
 * 4.2; x stays batch-major [n_meshes, nv, c]). */
int cfsd_swap_features_x(const float* x, const int32_t* batch_idx, const uint8_t* region_mask,
                         const int32_t* key, float* out, int out_dt, int bs, int nv, int c,
                         int n_meshes, int n_regions, void* stream);
/* SpiralDeblock forward with the Pool(up) fused into the gather (ABI 4.4;
 * model.py:80-82: x_up = Pool(xc, up) then SpiralConv(x_up) + ELU): the input
 * row of spiral position (r, s) is sum_k comp_val[(r*9+s)*3+k] *
 * xc[b, comp_col[(r*9+s)*3+k], :] -- the composite table of a uniform
 * 3-entry up matrix (topology.up_comp), summed ((0 + x0 v0) + x1 v1) + x2 v2
 * exactly as cfsd_spmm_uniform (bit-identical up-sampled rows); idx [rows, 9]
 * with idx[r][0] == r, and y_up (optional) receives the up-sampled input
 * [batch, rows, cin] the weight gradient reads.  xc [batch, n_coarse, cin],
 * y [batch, rows, cout], batch-major fp32.  Coarse layers only:
 * cfsd_spiral_conv_fwd_up_supported() says which. */
int cfsd_spiral_conv_fwd_up_supported(int batch, int rows, int seq, int cin, int cout);
int cfsd_spiral_conv_fwd_up(const float* xc, const int32_t* comp_col, const float* comp_val, const int32_t* idx,
                            const float* w, const float* bias, float* y, float* y_up, int batch, int n_coarse,
                            int rows, int seq, int cin, int cout, int act, void* stream);
/* The un-swapped batch of a swap_features: False configuration
 * (data_loading.py:38, 81-82: MeshCollater without a feature_swapper):
 * out[b] = x[batch_idx[b]], b < bs; out_dt = CFSD_DT_F32 [| CFSD_VM] (ABI 4.4).
 * Bit-exact copy; mesh indices clamped into [0, n_meshes). */
int cfsd_gather_meshes(const float* x, const int32_t* batch_idx, float* out, int out_dt, int bs, int nv,
                       int c, int n_meshes, void* stream);

/* Spectral augmentation blend (utils.py:244-267, data_loading.py:359-364):
 * with s1 = U^T x1, s2 = U^T x2 [pairs, k, c] (U: the k smallest Laplacian
 * eigenvectors), s4[p,j,:] = s1 + values[p,j]*(s2 - s1) for j < n_blend, else
 * s1; the augmented mesh is then U s4.  values [pairs, k] (spectral_interpolation:
 * N(0.5, 0.5) draws; spectral_combination: 0/1 selector). */
int cfsd_spectral_blend(const float* s1, const float* s2, const float* values, float* s4, int pairs,
                        int k, int c, int n_blend, void* stream);

/* Dataset normalisation, (x - mean) / std with per-vertex statistics
 * (data_loading.py:259-260; mean/std [nv, c] from norm.pt): x, out
 * [n_meshes, nv, c] (may alias).  Same two IEEE roundings as torch: bit-exact. */
int cfsd_normalize(const float* x, const float* mean, const float* std, float* out, int n_meshes,
                   int nv, int c, void* stream);

/* ---------------------------------------------------------------- dense layers
 * nn.Linear of the latent bottleneck (model.py:114-124, 153-156, 167):
 *   y[i,n] = bias[n] + sum_k x[i,k] w[n,k]      x [m,k], w [n,k], y [m,n]
 * Long reductions are split across workgroups through `workspace`
 * (cfsd_linear_workspace(m,k,n) bytes; may be 0 -> NULL allowed). */
size_t cfsd_linear_workspace(int m, int k, int n);
int cfsd_linear_fwd(const float* x, const float* w, const float* bias, float* y, float* workspace,
                    size_t workspace_bytes, int m, int k, int n, void* stream);
/* Linear backward: dx = dy.w (times elu'(elu_y) when elu_y [m,k] != NULL; added
 * to dx when accumulate != 0), dw = dy^T.x, db = sum_i dy.  dx/dw/db may be NULL. */
int cfsd_linear_bwd(const float* x, const float* w, const float* dy, const float* elu_y, float* dx,
                    float* dw, float* db, float* workspace, size_t workspace_bytes, int m, int k,
                    int n, int accumulate, void* stream);

/* Linear backward with a long output (the decoder Linear, dz = dh.W with
 * W [n][k], n = 4288): dW / db as cfsd_linear_bwd and, in the SAME launch,
 * dx as cfsd_linear_bwd_split_parts(n) partial products over 64-row slices of
 * W, dx_parts [parts][m][k] (summed by cfsd_latent_bwd_parts, slice order).
 * m <= 16, k <= 128. */
int cfsd_linear_bwd_split_parts(int n);
int cfsd_linear_bwd_split(const float* x, const float* w, const float* dy, float* dx_parts,
                          float* dw, float* db, int m, int k, int n, void* stream);

/* The step's whole bottleneck backward in ONE launch (ABI 4.8; 4.12: the
 * exchange workspace, the sticky error word): the Pool(up)
 * transpose of the coarsest Deblock (model.py:172-173; CSR up_ptr/up_col/
 * up_val in plain per-row order over the fine-level gradient g [batch][n_up]
 * [cup], batch-major), the decoder Linear backward (dh.W with W = wd
 * [nd][latent], nd = coarse vertices x cup; dwd / dbd; dz as the partial
 * products of cfsd_linear_bwd_split, kept in `exchange`), the latent head
 * backward (cfsd_latent_bwd_parts: mulv, eps, dlat -> dmulv) and the encoder
 * Linear backward (cfsd_linear_bwd with x = xe [batch][ke], w = we [ne][ke],
 * dy = dmulv; dxe (x elu'(elu_y) when elu_y != NULL), dwe, dbe).  Workgroups
 * of the later stages wait on device counters for the earlier ones (only ever
 * on workgroups of lower index) and read the values they wait for from
 * `exchange` (cfsd_bottleneck_bwd_exchange_floats(batch, latent, nd, ne)
 * device floats, contents unspecified: each 128-B line is written by ONE
 * workgroup); `sync` is 608 device int32 (19 counters and flags, one 128-B
 * line each) that must be zero before the first call and are left zero by
 * every call -- except sync[CFSD_BN_SYNC_ERR], a sticky word a wait that
 * timed out sets (the values are then wrong: the caller must check it and
 * refuse the step).  Same values bit for bit as spmm + linear_bwd_split +
 * latent_bwd_parts + linear_bwd, except that dh itself is never stored.
 * batch <= 16, latent <= 128, cup a multiple of 64, nd <= 5120, ne =
 * (is_vae ? 2 : 1) x latent <= 160. */
#define CFSD_BN_SYNC_ERR 65
size_t cfsd_bottleneck_bwd_exchange_floats(int batch, int latent, int nd, int ne);
int cfsd_bottleneck_bwd(const int32_t* up_ptr, const int32_t* up_col, const float* up_val, const float* g,
                        int n_up, int cup, const float* z, const float* wd, float* exchange, float* dwd,
                        float* dbd, int nd, const float* mulv, const float* eps, const float* dlat,
                        float* dmulv, int train, int is_vae, int sigmoid, const float* xe, const float* we,
                        const float* elu_y, float* dxe, float* dwe, float* dbe, int ke, int ne, int accumulate,
                        int32_t* sync, int batch, int latent, void* stream);

/* ---------------------------------------------------------------- losses
 * compute_mse_loss + _compute_laplacian_regularizer (model_manager.py:333-349,
 * utils.py:153-165) fused.  Pass 1 computes, per (b,v), Lx = sum_k L[v,k] pred[b,k,:]
 * (CSR of the random-walk Laplacian, per-row order = COO order), stores the
 * unit vector Lx/|Lx| in unit_lx [batch, nv, c] and writes per-block partial
 * sums {sum (pred-gt)^2, sum |Lx|} to partials[2*nblocks] (nblocks from
 * cfsd_recon_lap_blocks).  Pass 2 writes the gradient of
 *   w_rec * mse + w_lap * sum|Lx| / (nv*batch)
 * w.r.t. pred into dpred using the transpose CSR (lt_*). */
int cfsd_recon_lap_blocks(int batch, int nv);
int cfsd_recon_lap_fwd(const float* pred, const float* gt, const int32_t* l_ptr,
                       const int32_t* l_col, const float* l_val, float* unit_lx, float* partials,
                       int batch, int nv, int c, void* stream);
int cfsd_recon_lap_bwd(const float* pred, const float* gt, const float* unit_lx,
                       const int32_t* lt_ptr, const int32_t* lt_col, const float* lt_val,
                       float* dpred, int batch, int nv, int c, float w_rec, float w_lap,
                       void* stream);
/* cfsd_recon_lap_bwd with cfsd_loss_finalize folded into its last workgroup
 * (same arguments as both; the partials were completed by the preceding
 * cfsd_recon_lap_fwd on the stream): one launch less per train step. */
int cfsd_recon_lap_bwd_finalize(const float* pred, const float* gt, const float* unit_lx,
                                const int32_t* lt_ptr, const int32_t* lt_col, const float* lt_val,
                                float* dpred, int batch, int nv, int c, float w_rec, float w_lap,
                                const float* partials, int nblocks, const float* terms, float* out,
                                float* acc, float w_kl, float w_lc, void* stream);
/* The three loss passes with pred / gt / unit_lx / dpred in one layout, dt =
 * CFSD_DT_F32 [| CFSD_VM] (ABI 4.2: the fp32 step's vertex-major level-0
 * tensors).  Same values; the loss partial sums run over the storage order,
 * so the reduced losses may differ in the last bits between layouts. */
int cfsd_recon_lap_fwd_x(const float* pred, const float* gt, const int32_t* l_ptr,
                         const int32_t* l_col, const float* l_val, float* unit_lx, float* partials,
                         int batch, int nv, int c, int dt, void* stream);
int cfsd_recon_lap_bwd_x(const float* pred, const float* gt, const float* unit_lx,
                         const int32_t* lt_ptr, const int32_t* lt_col, const float* lt_val,
                         float* dpred, int batch, int nv, int c, float w_rec, float w_lap, int dt,
                         void* stream);
int cfsd_recon_lap_bwd_finalize_x(const float* pred, const float* gt, const float* unit_lx,
                                  const int32_t* lt_ptr, const int32_t* lt_col, const float* lt_val,
                                  float* dpred, int batch, int nv, int c, float w_rec, float w_lap,
                                  const float* partials, int nblocks, const float* terms, float* out,
                                  float* acc, float w_kl, float w_lc, int dt, void* stream);

/* Latent head, forward (model.py:146-160, 184-188; model_manager.py:352-393).
 * mulv [batch, 2*latent] = [logvar | mu] when is_vae (the two encoder Linears
 * stacked, logvar = en_layers[-2], mu = en_layers[-1]), else mu [batch, latent].
 * z = mu + eps*exp(0.5*logvar) (train && is_vae), sigmoid(mu) (!is_vae && sigmoid),
 * else mu.  KL and the latent-consistency hinge for the swapped region
 * [key*region_size, +region_size) (key: device scalar; bs = sqrt(batch)).
 * Writes z [batch, latent]; terms[2] = {kl, lc}; and the head's own gradient
 * parts dlat [batch, 3*latent] = {w_lc*dLC/dz | w_kl*dKL/dmu | w_kl*dKL/dlogvar}.
 * Single workgroup holding z and the pair distances in LDS: needs
 * 4 (batch*latent + 4*npairs*bs) bytes <= 159 KB (batch 256 at latent 75:
 * 105 KB); larger shapes return CFSD_EINVAL. */
int cfsd_latent_fwd(const float* mulv, const float* eps, const int32_t* key, float* z,
                    float* dlat, float* terms, int batch, int latent, int region_size, int train,
                    int is_vae, int sigmoid, float w_kl, float w_lc, float eta1, float eta2,
                    void* stream);
/* (ABI 4.5) cfsd_latent_fwd followed by the decoder Linear (model.py:167-168)
 * y [batch, n] = z w^T + bias, w [n, latent], in ONE launch: z, dlat and y are
 * bit-identical to cfsd_latent_fwd + cfsd_linear_fwd(z, w, bias, y, batch,
 * latent, n), terms[] included.  _supported: latent <= 80 and the LDS of z,
 * the pair distances and a 32-row W slice <= 159 KB. */
int cfsd_latent_linear_fwd_supported(int batch, int latent, int n);
int cfsd_latent_linear_fwd(const float* mulv, const float* eps, const int32_t* key, float* z,
                           float* dlat, float* terms, int batch, int latent, int region_size,
                           int train, int is_vae, int sigmoid, float w_kl, float w_lc, float eta1,
                           float eta2, const float* w, const float* bias, float* y, int n,
                           void* stream);
/* Latent head, backward: dmulv (same layout as mulv) from dz_dec (gradient of
 * the decoder input) + dlat.  z is only read for the sigmoid AE variant. */
int cfsd_latent_bwd(const float* mulv, const float* eps, const float* z, const float* dz_dec,
                    const float* dlat, float* dmulv, int batch, int latent, int train, int is_vae,
                    int sigmoid, void* stream);
/* cfsd_latent_bwd with dz_dec given as n_parts partial products
 * [n_parts][batch][latent] (from cfsd_linear_bwd_split), summed in part order. */
int cfsd_latent_bwd_parts(const float* mulv, const float* eps, const float* z,
                          const float* dz_parts, int n_parts, const float* dlat, float* dmulv,
                          int batch, int latent, int train, int is_vae, int sigmoid, void* stream);
/* Reduce the recon partials + latent terms into out[5] = {rec, kl, lc, lap, tot}
 * (tot = rec + w_kl*kl + w_lc*lc + w_lap*lap, model_manager.py:308-312) and,
 * when acc != NULL, add them to acc[0..4] and 1 to acc[5] (per-epoch sums on
 * device: no per-step host sync, unlike the reference's 7 .item() calls). */
int cfsd_loss_finalize(const float* partials, int nblocks, const float* terms, float* out,
                       float* acc, int batch, int nv, int c, float w_kl, float w_lc, float w_lap,
                       void* stream);

/* ---------------------------------------------------------------- optimiser
 * torch.optim.Adam step (model_manager.py:69-72, 316) over one flat fp32
 * parameter buffer.  `step` is a device int32 holding the 1-based step number
 * t used for the bias corrections (advanced by cfsd_step_begin).  With
 * param_bf16 != NULL (8-B aligned) the updated parameters are also written
 * there as bf16 (the weight shadow the bf16 kernels read; may be NULL). */
int cfsd_adam(float* param, const float* grad, float* m, float* v, const int32_t* step, size_t n,
              float lr, float beta1, float beta2, float eps, float weight_decay,
              uint16_t* param_bf16, void* stream);

/* cfsd_scale(grad, n, grad_scale) then cfsd_adam in ONE launch (ABI 4.7): the
 * data-parallel step's 1/world averaging after the gradient all-reduce (SUM)
 * folded into the update (model_manager.py:316 on the averaged gradient).
 * `grad` receives the scaled gradient; same values bit for bit as the two
 * launches. */
int cfsd_adam_scaled(float* param, float* grad, float* m, float* v, const int32_t* step, size_t n,
                     float grad_scale, float lr, float beta1, float beta2, float eps,
                     float weight_decay, uint16_t* param_bf16, void* stream);

/* Per-step device bookkeeping (graph-replayable, no host input):
 * t = ++*counter; key = hash(seed, t) % n_regions (replaces random.choice,
 * swap_batch_transform.py:26); eps[n_eps] ~ N(0,1) (replaces randn_like,
 * model.py:187); the batch of MeshLoader(shuffle=True, drop_last=True)
 * (data_loading.py:40-48): with bt = (t-1) % n_batches, epoch = (t-1) / n_batches,
 *   j_q = shuffle ? P_epoch(bt*bs + q) : bt*bs + q,   batch_idx[q] = perm ? perm[j_q] : j_q
 * where P_epoch is a keyed permutation of [0, n_items) drawn from (seed, epoch)
 * (a fresh order every epoch; n_batches*bs <= n_items, the tail is dropped) and
 * perm (n_items entries, optional) maps positions to dataset rows (e.g. a
 * rank's shard); ++*adam_step (the Adam bias-correction step of this iteration).
 * Any of eps/key/batch_idx/adam_step may be NULL. */
int cfsd_step_begin(int32_t* counter, unsigned long long seed, float* eps, int n_eps,
                    int32_t* key, int n_regions, int32_t* batch_idx, int bs, int n_batches,
                    const int32_t* perm, int n_items, int shuffle, int32_t* adam_step,
                    void* stream);

/* F.elu backward written from the ELU output (model.py:68,84 autograd):
 * dx = dy * (y > 0 ? 1 : y + 1).  dx may alias dy. */
int cfsd_elu_bwd(const float* dy, const float* y, float* dx, size_t n, void* stream);

/* Element-wise y *= alpha (gradient averaging after an all-reduce). */
int cfsd_scale(float* y, size_t n, float alpha, void* stream);

/* ---------------------------------------------------------------- bf16 path
 * Mixed-precision variants (BASELINE.json configs C3/C5: bf16 activations and
 * weights, fp32 accumulation, fp32 master weights + Adam).  Each activation /
 * gradient operand carries its storage type (CFSD_DT_F32 / CFSD_DT_BF16);
 * the engine's bf16 mode keeps the level-0/1 tensors in bf16 and the coarse
 * levels + bottleneck in fp32.  Same arithmetic as the fp32 entry points
 * above (model.py:27-55 and autograd), products in bf16, sums in fp32.
 * 32/64-channel layers need x bf16 and the bf16 weight shadow `w_bf16`
 * ([cout, seq*cin], from cfsd_adam/cfsd_cast); the xyz layers use the fp32
 * `w` (input conv: x fp32 -> y bf16; output conv: x bf16 -> y fp32).
 *
 * The same entry points take the fp32 step's VERTEX-MAJOR operands (ABI 4.1,
 * the reference's fp32 arithmetic with the level-0/1 tensors stored
 * [nv][batch][c], batch % 16 == 0): a 32 -> 32/64 layer with x_dt =
 * CFSD_DT_F32 | CFSD_VM runs the fp32 vertex-major MFMA kernels with the fp32
 * `w` (y fp32, either layout; same products in the same order as
 * cfsd_spiral_conv_fwd, bit-identical outputs), and the xyz layers accept
 * fp32 operands in either layout. */
int cfsd_spiral_conv_fwd_x(const void* x, int x_dt, const int32_t* idx, const float* w,
                           const uint16_t* w_bf16, const float* bias, void* y, int y_dt, int batch,
                           int vsrc, int rows, int seq, int cin, int cout, int act, void* stream);
/* dx (bf16) of a 32/64-channel layer; dpre bf16 or fp32; elu_y bf16 or NULL.
 * dx_dt = CFSD_DT_BF16 [| CFSD_VM] (the layout of dx and elu_y). */
int cfsd_spiral_conv_bwd_data_x(const void* dpre, int dpre_dt, const int32_t* inv_ptr,
                                const int32_t* inv_row, const int32_t* inv_head,
                                const uint16_t* w_bf16, const uint16_t* elu_y, uint16_t* dx,
                                int dx_dt, int batch, int vsrc, int rows, int seq, int cin,
                                int cout, void* stream);
/* The same dx through the FLAT inverse list (topology.inverse_flat: per
 * source vertex the spiral positions p = r*seq + s naming it, ascending,
 * -1 padded to flat_width in {8, 12, 16, 20}): one MFMA per entry, exact
 * products (no bf16 rounding of per-slot row sums).  Vertex-major dpre / dx /
 * elu_y, batch % 16 == 0, 32 -> 32/64 channels (the level-0/1 Deblocks).
 * dx_dt = CFSD_DT_BF16 | CFSD_VM: `w` is the bf16 shadow, elu_y bf16, dpre
 * bf16 or fp32; dx_dt = CFSD_DT_F32 | CFSD_VM (ABI 4.1, the fp32 step): `w`,
 * elu_y and dpre fp32 -- dx[u] = elu'(elu_y[u]) * sum over the list of
 * W_s^T dpre[r] in list order (IndexSelectBackward's visiting order). */
int cfsd_spiral_conv_bwd_data_flat(const void* dpre, int dpre_dt, const int32_t* inv_flat,
                                   int flat_width, const void* w, const void* elu_y, void* dx,
                                   int dx_dt, int batch, int vsrc, int rows, int seq, int cin,
                                   int cout, void* stream);
/* dW/db (fp32): 32/64-channel layers (x bf16, dpre bf16/fp32; or x and dpre
 * fp32, each batch-major or vertex-major) and the xyz input layer (x fp32,
 * dpre bf16 or fp32).  dw == db == NULL defers the reduction
 * (cfsd_dw_reduce_batch item with fused = 2 for the bf16 32/64-channel kind,
 * 0 for fp32 x and for the input layer). */
size_t cfsd_spiral_conv_bwd_weight_x_workspace(int batch, int rows, int seq, int cin, int cout);
int cfsd_spiral_conv_bwd_weight_x(const void* x, int x_dt, const int32_t* idx, const void* dpre,
                                  int dpre_dt, float* dw, float* db, float* workspace,
                                  size_t workspace_bytes, int batch, int vsrc, int rows, int seq,
                                  int cin, int cout, void* stream);
/* Fused dx + dW of the xyz output layer (cout*seq <= 32) with x, elu_y, dx
 * bf16 (or all three fp32, ABI 4.1) and dpre fp32 (workspace:
 * cfsd_spiral_conv_bwd_workspace; deferred items use fused = 1).  x_dt's
 * storage type and CFSD_VM flag are those of x, elu_y and dx; dpre_dt =
 * CFSD_DT_F32 [| CFSD_VM]. */
int cfsd_spiral_conv_bwd_x(const void* x, int x_dt, const int32_t* idx, const float* dpre,
                           int dpre_dt, const int32_t* inv_ptr, const int32_t* inv_row, const int32_t* inv_head,
                           const float* w, const void* elu_y, void* dx, float* dw, float* db,
                           float* workspace, size_t workspace_bytes, int batch, int vsrc, int rows,
                           int seq, int cin, int cout, void* stream);
/* The same fused backward of the xyz output conv (32 -> 3) for VERTEX-MAJOR
 * x / elu_y / dx (fp32 or bf16) and fp32 dpre (ABI 4.2), batch % 16 == 0:
 * per source vertex the spiral transpose is one walk of its flat inverse
 * list (topology.inverse_flat, width 8/12/16/20), dx = W^T-products of the
 * folded 3-wide dpre, dW = folded dpre (x) x.  Same workspace, slab layout
 * and deferred kind (fused = 1) as cfsd_spiral_conv_bwd_x. */
int cfsd_spiral_conv_bwd_out_flat(const void* x, int x_dt, const int32_t* idx, const float* dpre,
                                  int dpre_dt, const int32_t* inv_flat, int flat_width, const float* w,
                                  const void* elu_y, void* dx, float* dw, float* db, float* workspace,
                                  size_t workspace_bytes, int batch, int vsrc, int rows, int seq, int cin,
                                  int cout, void* stream);
/* cfsd_spmm_csr with per-operand storage types (elu_y has y's type). */
int cfsd_spmm_csr_x(const int32_t* row_ptr, const int32_t* col, const float* val, const void* x,
                    int x_dt, const void* elu_y, void* y, int y_dt, int batch, int m, int n, int c,
                    void* stream);
/* Storage conversion fp32 <-> bf16 (round to nearest even), n elements. */
int cfsd_cast(const void* src, int src_dt, void* dst, int dst_dt, size_t n, void* stream);

/* ---------------------------------------------------------------- evaluation
 * Replaces ModelManager.compute_vertex_errors (model_manager.py:395-400) and
 * the per-mesh reduction of Tester.reconstruction_errors (test.py:280-301):
 * out, gt [batch, nv, 3]; mean/std [nv, 3] (both NULL = no un-normalisation,
 * else u = x*std + mean as Tester._unnormalize_verts, test.py:81-84);
 *   err[b, v]  = sqrt(sum_c (u_out - u_gt)^2) * to_mm        (may be NULL)
 *   l1[b, v]   = sum_c |u_out - u_gt|  (the per-vertex L1 parity metric; may be NULL)
 *   mesh_mean[b] = mean_v err[b, v]  (fixed-order reduction; needs err; may be NULL). */
int cfsd_vertex_errors(const float* out, const float* gt, const float* mean, const float* std,
                       float* err, float* l1, float* mesh_mean, int batch, int nv, float to_mm,
                       void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CFSD_H */
