// lrl_gemm.h — LDS-tiled fp32 MFMA GEMM for the PPO minibatch update (gfx950).
//
// C(m, n) = sum_k A(m, k) B(k, n) on v_mfma_f32_32x32x2_f32 (exact fp32, k-ordered FMA chain), with
// the three operand layouts an MLP's forward / backward-data / weight-gradient products need:
//   forward       Y[b][o]  = X[b][i] W[o][i]        A k-contiguous, B k-contiguous   (+bias, ELU)
//   backward-data dX[b][i] = dY[b][o] W[o][i]       A k-contiguous, B n-contiguous   (* ELU'(X))
//   weight grad   dW[o][i] = dY[b][o] X[b][i]       A m-contiguous, B n-contiguous   (split over b)
// The batch dimension of a k-contiguous A (the rows of X) and of an n-contiguous B (the rows of X in
// the weight gradient) may be gathered through an int64 row list — the minibatch indices of
// RolloutStorage.mini_batch_generator (rollout_storage.py:100-137) — so the minibatch is never copied.
//
// Three kernels behind one launcher (gemm_launch picks by shape):
//  * LDS-DMA (NT / NN, every tile interior, float4-aligned operands): 64 x 64 tile, 16-k slices land in a
//    3-stage LDS ring straight from global memory (global_load_lds_dwordx4, counted vmcnt waits, swizzled
//    images read with ds_read_b128), two accumulators per wave;
//  * thin (NT / NN, N <= 32, k = 512 / 1024): op(B) kept in registers per k-quarter, A streamed a block
//    ahead, quarter sums added in wave order;
//  * register-staged (everything else, incl. the split-k weight gradients): a workgroup (4 waves) owns a
//    BM x BN tile (128 / 64 wide, 32 for thin layers); 16-k slices stage through LDS k-major so each MFMA
//    operand is one ds_read_b32 per lane; the next slice is prefetched into registers while the current one
//    is consumed; the tile order is XCD-aware (consecutive tiles on one XCD share the A row block).
// Every path sums k in a fixed order: results are deterministic run to run.
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define LRL_GHD __host__ __device__
#else
#define LRL_GHD
#endif

namespace lrl {

enum GemmEpi : int {
  EPI_STORE = 0,     // C = acc
  EPI_BIAS = 1,      // C = acc + bias[n]
  EPI_BIAS_ELU = 2,  // C = elu(acc + bias[n])
  EPI_DELU = 3,      // C = acc * elu'(aux[m][n])  (aux = ELU output of the layer input: elu' = aux > 0 ? 1 : aux + 1)
  EPI_PARTIAL = 4,   // split-k partial: C + split * part_stride (+ bias-gradient partial of A's columns)
};

struct GemmP {
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  const float* aux;
  const int64_t* a_rows;  // k-contiguous A: row list for m (nullptr = identity)
  const int64_t* b_rows;  // n-contiguous B: row list for k (nullptr = identity)
  float* bias_part;       // EPI_PARTIAL: [splits][groups][M] partial sums over k of A(m, k), or nullptr
  int M, N, K;
  int splits, kps;        // k range of split s: [s*kps, min(K, (s+1)*kps))
  int avec, bvec;         // staging access width (4/2/1 floats), set by gemm_launch from the alignment
  int groups;             // set by gemm_launch
  int64_t lda, ldb, ldc, ld_aux;
  int64_t ga, gb, gc, gbias, gaux;  // per-group element offsets
  int64_t part_stride;              // EPI_PARTIAL: elements between split slices of C ([split][group][M][N])
  // pre-split B (x6p kernel, NT / NN): hi / mid / lo bf16 planes of op(B) in [n][k] form (x6_planes_launch), k padded
  // to bpl_ld (a multiple of 16, zero past K); plane pl of group g at bpl + pl * bpl_ps + g * gbp.  nullptr: B is read
  // as fp32 from `B` by the other kernels
  const uint16_t* bpl;
  int64_t bpl_ld, bpl_ps, gbp;
};

// One weight matrix to split into planes: W is [rows][cols] (ldw) per group (gsrc elements apart); op(B) in [n][k]
// form is W itself (trans = 0: n = row, k = col — the forward's B) or its transpose (trans = 1: n = col, k = row — the
// backward-data B).  dst receives [3][groups][n][kp] bf16 (kp = k rounded up to 16; the padding is zero).
struct PlaneJob {
  const float* W;
  int64_t ldw, gsrc;
  int rows, cols, trans, groups;
  uint16_t* dst;
};
constexpr int MAX_PLANE_JOBS = 8;
LRL_GHD inline int plane_kp(const PlaneJob& j) { return ((j.trans ? j.rows : j.cols) + 15) / 16 * 16; }
LRL_GHD inline int plane_n(const PlaneJob& j) { return j.trans ? j.cols : j.rows; }
LRL_GHD inline int64_t plane_elems(const PlaneJob& j) { return 3ll * j.groups * plane_n(j) * plane_kp(j); }
// Split every job's matrix into its planes (one launch for up to MAX_PLANE_JOBS jobs).
int x6_planes_launch(const PlaneJob* jobs, int n, void* stream);
// false when LRL_GEMM_X6P=0 (no planes: every product reads fp32 B)
bool gemm_x6p_enabled();
// Point p's pre-split B at job j's planes.
inline void gemm_use_planes(GemmP& p, const PlaneJob& j) {
  p.bpl = j.dst;
  p.bpl_ld = plane_kp(j);
  p.gbp = (int64_t)plane_n(j) * plane_kp(j);
  p.bpl_ps = p.gbp * j.groups;
}

// layout: bit0 = A m-contiguous, bit1 = B n-contiguous
enum GemmLayout : int { GEMM_NT = 0, GEMM_NN = 2, GEMM_TN = 3 };

// Enqueue C = op(A, B) for `groups` independent problems of the same shape.  Returns 0 or a negative
// lrl error code (bad shape / unsupported layout).
int gemm_launch(const GemmP& p, int layout, int epi, int groups, void* stream);

// 1 when this thread's last gemm_launch ran the x6p kernel (test entry point)
int gemm_last_path();

// How a weight-gradient product (reduction over K rows, `groups` problems) is split: the split count.
int gemm_pick_splits(int M, int N, int K, int groups);

}  // namespace lrl
