// All-pairs L2 retrieval: top-k gallery items and the rank of the positive.
//
// Reference (inference.py:30-69, utils.py:42): per query,
//   d_i = || q - g_i + 1e-6 ||_2   (nn.PairwiseDistance(p=2, eps=1e-6))
//   topk(N, largest=False) -> position of the positive; topk(k) -> top-k list.
// Here all queries are processed at once and the order is made total and
// exact: distances are EVALUATED in f64 from the f32 features and sorted by
// (distance, gallery index) — the oracle's definition (oracle/retrieval.py).
//
//  1. knn_scan_kernel (MFMA): for a (query tile x gallery chunk) workgroup,
//     stream gallery tiles, compute approximate squared distances
//     |q|^2 + |g|^2 - 2 q.g with bf16 (or exact-f32) MFMA and
//       * keep, per query, the T smallest approximate values of the chunk
//         (threshold filter -> rare insertions into a per-query register list),
//       * count items certainly closer than the positive (approx < lo_q) and
//         queue the uncertain ones (lo_q <= approx <= hi_q) for exact checks,
//     where [lo_q, hi_q] = d_pos^2 -/+ eps_q and eps_q bounds the approximation
//     error of the squared distance;
//  2. knn_merge_kernel: exact f64 distances of the S*T candidates of a query,
//     top-k by (distance, index), plus a verification flag if a chunk list
//     could have dropped a true top-k item (then the host reruns that query
//     with an exhaustive exact scan);
//  3. knn_uncertain_kernel: exact checks of the queued uncertain items.
//
// Error bound of the approximate squared distance |q|^2 + |g|^2 - 2 q.g
// (norms in f32 from the f32 rows, the dot product from the compute copies):
// bf16 rounding of each operand is relative <= 2^-8, so each product is off by
// <= (2^-7 + 2^-16)|q_i g_i| and the dot by <= 2^-7 sum|q_i g_i| <= 2^-7 |q||g|
// (Cauchy-Schwarz); products of bf16 are exact in f32 and the f32 accumulation
// adds < 2^-13 |q||g| for D <= 4096.  Hence |err(d^2)| <= rel |q| |g|max + 1e-3
// with rel = 2^-6 + 2^-12 (bf16) or 2^-14 (exact-f32 MFMA); every decision
// that could depend on the approximation is re-made in f64.
#include <utility>
#include <vector>

#include "common.h"
#include "../../include/artsbir.h"

namespace artsbir {

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4r;
#define ROOB 0x80000000u

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rrsrc(const void* base, long long bytes) {
  if (bytes > 0x7fffffffLL) bytes = 0x7fffffffLL;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 rload(__amdgpu_buffer_rsrc_t r, unsigned off) {
  u32x4r v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

template <typename T> struct RM;
template <> struct RM<bf16> {
  static constexpr int EPC = 8;
  __device__ __forceinline__ static void mma(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(&a),
                                                  *reinterpret_cast<const bf16x8*>(&b), acc, 0, 0, 0);
  }
};
template <> struct RM<float> {
  static constexpr int EPC = 4;
  __device__ __forceinline__ static void mma(f32x4& acc, const uint4& a, const uint4& b) {
    const float* fa = reinterpret_cast<const float*>(&a);
    const float* fb = reinterpret_cast<const float*>(&b);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[e], fb[e], acc, 0, 0, 0);
  }
};

// ---------------------------------------------------------------- helpers
// squared norm of each f32 row, and the compute-dtype copy of the row.
// normalize (cosine metric): the row is first scaled by 1/max(|x|, 1e-8) (|x| in
// f64), so the L2 scan of the unit rows orders by 1 - cos (|a-b|^2 = 2 - 2 cos)
__device__ __forceinline__ float row_scale(const float* r, int D, int lane, int normalize) {
  if (!normalize) return 1.f;
  double s = 0.0;
  for (int d = lane; d < D; d += 64) s += (double)r[d] * (double)r[d];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  return (float)(1.0 / fmax(sqrt(s), 1e-8));
}

// Rows whose columns allow 16-B loads are read 8 consecutive columns per lane
// (columns lane*8 + 512 j + i); rows_prep and rows_prep_aug both sum |x|^2 in
// that order then, so the two give bit-identical norms (the two scans must
// see the same d2); other rows column-strided per lane, in both.
__device__ __forceinline__ bool row_vec_ok(const float* r, int D) {
  return (D & 3) == 0 && (reinterpret_cast<unsigned long long>(r) & 15) == 0;
}
__device__ __forceinline__ void row_load8(const float* r, int D, int d0, float sc, float* v) {
  if (d0 + 8 <= D) {
    const float4 a = *reinterpret_cast<const float4*>(r + d0);
    const float4 b = *reinterpret_cast<const float4*>(r + d0 + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = d0 + j < D ? r[d0 + j] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] *= sc;
}

template <typename T>
__global__ void rows_prep_kernel(const float* __restrict__ x, int n, int D, float* __restrict__ sq, T* __restrict__ xc,
                                 int ldc, int normalize) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (row >= n) return;
  const float* r = x + (long long)row * D;
  const float sc = row_scale(r, D, lane, normalize);
  float s = 0.f;
  if (row_vec_ok(r, D)) {
    for (int d0 = lane * 8; d0 < ldc; d0 += 512) {
      float v[8];
      row_load8(r, D, d0, sc, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s = fmaf(v[j], v[j], s);  // explicit fma: the same rounding in both kernels
        if (xc && d0 + j < ldc) xc[(long long)row * ldc + d0 + j] = from_f<T>(v[j]);
      }
    }
  } else {
    for (int d = lane; d < ldc; d += 64) {  // the compute copy is zero-padded to ldc columns
      const float v = d < D ? r[d] * sc : 0.f;
      s = fmaf(v, v, s);
      if (xc) xc[(long long)row * ldc + d] = from_f<T>(v);
    }
  }
  s = warp_sum(s);
  if (lane == 0) sq[row] = s;
}

// exact ||q - g + eps|| in f64 (one wave)
__device__ __forceinline__ double exact_l2(const float* q, const float* g, int D, int lane) {
  double s = 0.0;
  for (int d = lane; d < D; d += 64) {
    const double t = ((double)q[d] - (double)g[d]) + 1e-6;
    s += t * t;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  return sqrt(s);
}

// Exact ordering key of (q, g) in f64 (one wave; all lanes return it):
//   metric 0  ||q - g + 1e-6||                                 nn.PairwiseDistance(p=2, eps=1e-6), utils.py:42
//   metric 1  1 - q.g / (max(|q|, 1e-8) max(|g|, 1e-8))        cosine_distance, utils.py:31-40
//             (nn.CosineSimilarity(dim=1, eps=1e-8): each norm clamped separately)
__device__ __forceinline__ double exact_key(const float* q, const float* g, int D, int lane, int metric) {
  if (metric == 0) return exact_l2(q, g, D, lane);
  double dot = 0.0, qq = 0.0, gg = 0.0;
  for (int d = lane; d < D; d += 64) {
    const double a = q[d], b = g[d];
    dot += a * b;
    qq += a * a;
    gg += b * b;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    dot += __shfl_xor(dot, o, 64);
    qq += __shfl_xor(qq, o, 64);
    gg += __shfl_xor(gg, o, 64);
  }
  return 1.0 - dot / (fmax(sqrt(qq), 1e-8) * fmax(sqrt(gg), 1e-8));
}

// the scan-domain squared distance of an exact key: d^2 itself for L2; for the
// cosine metric the scan runs on unit rows where d^2 = 2 key (the deviation of
// the f32 unit rows' norms from 1 is folded into the per-query eps, knn_qeps)
__device__ __forceinline__ double key_d2(double key, int metric) { return metric ? 2.0 * key : key * key; }

// per-query bound of |approx d^2 - scan-domain exact d^2|: rel |q| max|g| + 1e-3,
// plus for the cosine metric 2 (|1 - |q|^2| + max(gmax - 1, 1 - gmin)), the room
// between 2 key and |q^|^2 + |g^|^2 - 2 q^.g^ of the normalised f32 rows
__device__ __forceinline__ double query_eps(float qsq, float gmax, float gmin, float rel, int metric) {
  double e = rel * sqrt((double)qsq * gmax) + 1e-3;
  if (metric) e += 2.0 * (fabs(1.0 - (double)qsq) + fmax((double)gmax - 1.0, 1.0 - (double)gmin));
  return e;
}

// d_pos^2 (exact, f64) and the uncertainty band of every query
__global__ void knn_band_kernel(const float* __restrict__ q, const float* __restrict__ g, const long long* __restrict__ pos,
                                long long g_base, long long n_g, const float* __restrict__ qsq, float gsq_max, int nq, int D,
                                float rel, double* __restrict__ dpos, float* __restrict__ lo, float* __restrict__ hi,
                                int metric, const float* __restrict__ qeps) {
  const int lane = threadIdx.x & 63;
  const int qi = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (qi >= nq) return;
  const long long p = pos[qi];
  const double eps = qeps ? (double)qeps[qi] : rel * sqrt((double)qsq[qi] * gsq_max) + 1e-3;
  if (p < g_base || p >= g_base + n_g) {
    // positive not in this shard: the caller provides dpos from its owner
    if (lane == 0) {
      const double d = dpos[qi];
      lo[qi] = d >= 0 ? (float)(key_d2(d, metric) - eps) : -1.f;
      hi[qi] = d >= 0 ? (float)(key_d2(d, metric) + eps) : -1.f;
    }
    return;
  }
  const double d = exact_key(q + (long long)qi * D, g + (p - g_base) * D, D, lane, metric);
  if (lane == 0) {
    dpos[qi] = d;
    lo[qi] = (float)(key_d2(d, metric) - eps);
    hi[qi] = (float)(key_d2(d, metric) + eps);
  }
}

__global__ void knn_band_from_dpos_kernel(const double* __restrict__ dpos, const float* __restrict__ qsq, float gsq_max,
                                          int nq, float rel, float* __restrict__ lo, float* __restrict__ hi) {
  const int qi = blockIdx.x * blockDim.x + threadIdx.x;
  if (qi >= nq) return;
  const double eps = rel * sqrt((double)qsq[qi] * gsq_max) + 1e-3;
  const double d = dpos[qi];
  lo[qi] = d >= 0 ? (float)(d * d - eps) : -1.f;
  hi[qi] = d >= 0 ? (float)(d * d + eps) : -1.f;
}

// ------------------------------------------------------------ fused scan
struct KnnScanArgs {
  const void* q;  // [Nq][D] compute dtype
  const void* g;  // [Ng][D] compute dtype
  const float* qsq;
  const float* gsq;
  float gsq_max;  // knn_scan_v2: max |g|^2 (prefilter slack)
  const float* gsq_max_p;  // knn_scan_v2: if set, max |g|^2 read from device memory (one-call path, no host sync)
  const float* thr0;  // knn_scan_v2: optional per-query initial list threshold (see knn.py)
  unsigned* kb;       // knn_scan_v2: optional [Nq] shared k-th bound (kb_enc of an approx d2), atomicMin
  unsigned* hist;     // knn_scan_v2 (with kb): optional [Nq][HB_BINS] counts of published list items (zeroed)
  unsigned* hbase;    //   [Nq] the histogram's first bin key (0: not chosen yet; zeroed)
  int kq;             //   k of the final top-k (1..KT)
  float rel;          //   error bound factor of the approximate d2 (eps = rel |q| max|g| + 1e-3)
  int Nq, Ng, D;
  int tiles_per_chunk;
  int nchunks;
  const float* lo;  // rank band (nullptr: no rank)
  const float* hi;
  int* cnt;         // [Nq] items certainly closer than the positive
  int* unc;         // [unc_cap][2] (query, local gallery index); unc_n = unc + 2*unc_cap
  int unc_cap;
  float* cand_d;    // [Nq][nchunks][KT]
  int* cand_i;
};

constexpr int KT = 16;  // per (query, chunk) candidate list length

template <typename T>
__global__ void __launch_bounds__(256) knn_scan_kernel(KnnScanArgs a) {
  constexpr int EPC = RM<T>::EPC;
  constexpr int ES = sizeof(T);
  constexpr int BM = 128, BN = 128, BK = 8 * EPC;
  constexpr int A_BYTES = 8 * (BM + 1) * 16, B_BYTES = 8 * (BN + 1) * 16;
  constexpr int MAIN = 2 * (A_BYTES + B_BYTES);
  constexpr int LD = BN + 4;
  constexpr int EPI = BM * LD * 4;
  constexpr int SMEM = (MAIN > EPI ? MAIN : EPI);
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  __shared__ float s_gsq[BN];
  __shared__ float s_thr[BM];
  __shared__ int s_qn[BM];              // queued insertions per row this tile
  __shared__ float s_qd[BM][8];
  __shared__ int s_qi[BM][8];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int ntq = (a.Nq + BM - 1) / BM;
  // XCD-aware order: the hardware deals consecutive workgroups round-robin to
  // the 8 XCDs; remap so that the query tiles of one gallery chunk run on ONE
  // XCD at the same time and share each gallery tile through its L2 (instead
  // of every query tile fetching the whole chunk from HBM)
  int lid = (int)blockIdx.x;
  {
    const int nwg = (int)gridDim.x;
    if (nwg >= 8) {
      const int q8 = nwg / 8, r8 = nwg % 8, x = lid % 8;
      lid = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + lid / 8;
    }
  }
  const int chunk = lid / ntq;
  const int qt = lid % ntq;
  const int bm = qt * BM;
  const int tile0 = chunk * a.tiles_per_chunk;
  int ntiles = (a.Ng + BN - 1) / BN - tile0;
  if (ntiles > a.tiles_per_chunk) ntiles = a.tiles_per_chunk;
  if (ntiles <= 0) return;

  const __amdgpu_buffer_rsrc_t qr = rrsrc(reinterpret_cast<const T*>(a.q) + (long long)bm * a.D,
                                          (long long)(a.Nq - bm) * a.D * ES);
  // chunk-relative gallery descriptor keeps byte offsets in 31 bits for any N
  const long long g0 = (long long)tile0 * BN;
  const __amdgpu_buffer_rsrc_t gr = rrsrc(reinterpret_cast<const T*>(a.g) + g0 * a.D, (long long)(a.Ng - g0) * a.D * ES);
  const int lc = tid & 7, lr = tid >> 3;
  const int nk = a.D / BK;

  // the row owner (2 threads per row: t = 2r, 2r+1 scan one half each; 2r owns the list)
  const int my_row = tid >> 1, my_half = tid & 1;
  const bool owner = my_half == 0;
  const bool row_ok = bm + my_row < a.Nq;
  float lst_d[KT];
  int lst_i[KT];
#pragma unroll
  for (int i = 0; i < KT; ++i) { lst_d[i] = INFINITY; lst_i[i] = -1; }
  int closer = 0;
  const float lo = (a.lo && row_ok) ? a.lo[bm + my_row] : -1.f;
  const float hi = (a.lo && row_ok) ? a.hi[bm + my_row] : -1.f;
  const float qsq = row_ok ? a.qsq[bm + my_row] : 0.f;
  if (tid < BM) s_thr[tid] = INFINITY;

  uint4 ra[4], rb[4];
  for (int t = 0; t < ntiles; ++t) {
    const int bn = (tile0 + t) * BN;
    auto load_tiles = [&](int kt) {
      const int k0 = kt * BK;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = lr + 32 * i;
        ra[i] = rload(qr, (unsigned)((row * a.D + k0 + lc * EPC) * ES));
        const int gi = bn + row;
        rb[i] = rload(gr, gi < a.Ng ? (unsigned)(((gi - (int)g0) * a.D + k0 + lc * EPC) * ES) : ROOB);
      }
    };
    auto store_tiles = [&](int buf) {
      char* As = smem + buf * (A_BYTES + B_BYTES);
      char* Bs = As + A_BYTES;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        *reinterpret_cast<uint4*>(As + (lc * (BM + 1) + lr + 32 * i) * 16) = ra[i];
        *reinterpret_cast<uint4*>(Bs + (lc * (BN + 1) + lr + 32 * i) * 16) = rb[i];
      }
    };
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (tid < BN) s_gsq[tid] = (bn + tid < a.Ng) ? a.gsq[bn + tid] : INFINITY;
    load_tiles(0);
    store_tiles(0);
    __syncthreads();
    const int fr = lane & 15, fq = lane >> 4;
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) load_tiles(kt + 1);
      const char* As = smem + cur * (A_BYTES + B_BYTES);
      const char* Bs = As + A_BYTES;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int gq = kk * 4 + fq;
        uint4 af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const uint4*>(As + (gq * (BM + 1) + wm * 64 + i * 16 + fr) * 16);
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = *reinterpret_cast<const uint4*>(Bs + (gq * (BN + 1) + wn * 64 + j * 16 + fr) * 16);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) RM<T>::mma(acc[i][j], af[i], bfr[j]);
      }
      if (kt + 1 < nk) store_tiles(cur ^ 1);
      __syncthreads();
    }
    // stage q.g as f32, then each row is scanned by two threads (64 columns each)
    float* st = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) st[(wm * 64 + i * 16 + fq * 4 + r) * LD + wn * 64 + j * 16 + fr] = acc[i][j][r];
    if (tid < BM) s_qn[tid] = 0;
    __syncthreads();
    if (row_ok) {
      const float thr = s_thr[my_row];  // INF on the first tile: the owner rescans instead
      const float* srow = st + my_row * LD + my_half * 64;
      for (int c4 = 0; c4 < 64; c4 += 4) {
        const float4 s4 = *reinterpret_cast<const float4*>(srow + c4);
        const float sv[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = my_half * 64 + c4 + e;
          const float d2 = qsq + s_gsq[c] - 2.f * sv[e];
          if (d2 < thr && thr != INFINITY) {
            const int slot = atomicAdd(&s_qn[my_row], 1);
            if (slot < 8) { s_qd[my_row][slot] = d2; s_qi[my_row][slot] = bn + c; }
          }
          if (hi >= 0.f && bn + c < a.Ng) {
            if (d2 < lo) {
              ++closer;
            } else if (d2 <= hi) {
              const int k = atomicAdd(a.unc + 2 * a.unc_cap, 1);
              if (k < a.unc_cap) { a.unc[2 * k] = bm + my_row; a.unc[2 * k + 1] = bn + c; }
            }
          }
        }
      }
    }
    __syncthreads();
    // the owner merges the queued values into its sorted register list; if the
    // list was not yet full (first tile) or the queue overflowed, it rescans the
    // whole staged row instead
    if (owner && row_ok) {
      const int nq = s_qn[my_row];
      auto insert = [&](float x, int xi) {
#pragma unroll
        for (int i = 0; i < KT; ++i) {  // compare-swap down the sorted list
          const bool sw = x < lst_d[i] || (x == lst_d[i] && xi < lst_i[i] && lst_i[i] >= 0);
          const float td = lst_d[i];
          const int ti = lst_i[i];
          lst_d[i] = sw ? x : td;
          lst_i[i] = sw ? xi : ti;
          x = sw ? td : x;
          xi = sw ? ti : xi;
        }
      };
      if (nq > 8 || s_thr[my_row] == INFINITY) {
        const float* srow = st + my_row * LD;
        const float thr0 = s_thr[my_row];
        for (int c = 0; c < BN; ++c) {
          const float d2 = qsq + s_gsq[c] - 2.f * srow[c];
          if (d2 < thr0 && bn + c < a.Ng) insert(d2, bn + c);
        }
      } else {
        for (int k = 0; k < nq; ++k) insert(s_qd[my_row][k], s_qi[my_row][k]);
      }
      s_thr[my_row] = lst_d[KT - 1];
    }
    __syncthreads();
  }
  if (row_ok) {
    if (closer) atomicAdd(a.cnt + bm + my_row, closer);
    if (owner) {
      const long long o = ((long long)(bm + my_row) * a.nchunks + chunk) * KT;
#pragma unroll
      for (int i = 0; i < KT; ++i) {
        a.cand_d[o + i] = lst_d[i];
        a.cand_i[o + i] = lst_i[i];
      }
    }
  }
}

// ------------------------------------- register-resident scan (bf16, v2)
// One workgroup = 8 waves = 256 queries x one gallery chunk.  Each wave holds
// the MFMA A fragments of its 32 queries over the whole of D in registers
// (KB = Dp/16 uint4 per lane) and streams the chunk in 32-row gallery tiles
// that all 8 waves read from LDS: one v_mfma_f32_32x32x16_bf16 per k-block
// needs one ds_read_b128 (its B fragment) and no A traffic, and no tile is
// re-fetched per query tile of the workgroup.
//
// Gallery rows are stored AUGMENTED: [Ng][Dp + 8] bf16 whose columns Dp..Dp+1
// carry the f32 |g|^2 (artsbir_rows_prep_aug).  A 32-row tile is then one
// contiguous block of 32 * (2 Dp + 16) bytes, copied by LDS-DMA into a 3-stage
// ring, and the odd row pitch in 16-B slots (2 KB + 1) makes the B-fragment
// reads conflict-free (lanes r = 0..31 of a group hit slots r + const mod 16)
// with no swizzle.
//
// Epilogue per tile, in registers (32x32 accumulator: column = lane & 31 =
// gallery row, rows (e & 3) + 8 (e >> 2) + 4 (lane >> 5) = queries):
//   d2 = |q|^2 + |g|^2 - 2 q.g; any lane with d2 <= crit[row] (crit =
//   max(16th smallest of the chunk so far, rank band hi)) sends the wave into a
//   slow path that stages the tile's values in LDS, builds per-row hit masks by
//   ballot, counts "certainly closer" items by popcount and queues uncertain
//   ones; owner lanes (lane r < 32 owns row r) then insert their hits into a
//   sorted 16-entry register list.  Same candidate lists, counts and queue as
//   knn_scan_kernel (same d2 formula, same (value, index) order).
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((address_space(3))) void* r_lds_t;

// LDS-DMA of 16 B per lane to lds + 16 * lane (inline asm on purpose: the
// compiler does not track it, so it neither drains it before every ds_read nor
// at barriers; completion is counted by hand with rvm_wait).  M0 is written and
// restored inside the statement (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void rdma16(__amdgpu_buffer_rsrc_t r, char* lds, unsigned voff) {
  const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long long)(r_lds_t)lds);
  unsigned keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(base), "s"(r)
      : "memory");
}
template <int N>
__device__ __forceinline__ void rvm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void rvm_wait_n(int n) {
  switch (n) {
    case 1: rvm_wait<1>(); break;
    case 2: rvm_wait<2>(); break;
    case 3: rvm_wait<3>(); break;
    case 4: rvm_wait<4>(); break;
    case 5: rvm_wait<5>(); break;
    case 6: rvm_wait<6>(); break;
    case 7: rvm_wait<7>(); break;
    case 8: rvm_wait<8>(); break;
    case 9: rvm_wait<9>(); break;
    case 10: rvm_wait<10>(); break;
    default: rvm_wait<0>(); break;
  }
}

// order-preserving unsigned encoding of a float (atomicMin on the shared bound)
__device__ __forceinline__ unsigned kb_enc(float f) {
  const unsigned b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float kb_dec(unsigned u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}
// a list threshold every chunk may use: some chunk's k-th smallest approximate d2
// U >= the gallery's k-th smallest a_k, so U + 2 eps (+ rounding margin) >= the
// exact merge's cut a_k + 2 eps: no item at or above it can reach the top k
__device__ __forceinline__ float kb_bound(unsigned u, float eps) {
  const float v = kb_dec(u);
  return (v + 2.f * eps) * (1.f + 0x1p-18f) + 1e-3f;
}

// Per-query histogram of the approximate d2 of published list items: bins of
// 2^-7 octave (the float's exponent and top 7 mantissa bits), HB_BINS of them
// from a base key chosen once per query (atomicCAS, from the first chunk to
// publish: its kq-th smallest + 2 eps is the top bin).  A gallery item is
// counted at most once (each chunk publishes the list items it inserted since
// its previous exchange, once), so when the counts of bins <= b reach kq, at
// least kq distinct items have approx d2 < hb_edge(b): an upper bound of the
// gallery's kq-th smallest approx d2, exactly what kb holds (kb_bound).  Unlike
// one chunk's own kq-th smallest it tightens with everything every chunk has
// scanned so far: 570 -> ~130 items per query under the bound by mid-scan at
// C4 (1M x 512, randn rows).
constexpr int HB_BINS = 64;
__device__ __forceinline__ unsigned hb_key(float v) { return v > 0.f ? __float_as_uint(v) >> 16 : 0u; }
__device__ __forceinline__ int hb_bin(float v, unsigned base) {
  const unsigned kk = hb_key(v);
  return kk <= base ? 0 : (int)min(kk - base, (unsigned)HB_BINS);  // HB_BINS: above the top bin, not counted
}
__device__ __forceinline__ float hb_edge(unsigned base, int b) { return __uint_as_float((base + b + 1) << 16); }
// the smallest bin edge with >= kq counted items below it (+INF if none); the
// counts are read at agent scope (other XCDs' adds are not in this XCD's L2)
__device__ float hb_bound(const unsigned* hq, unsigned base, int kq) {
  unsigned cum = 0;
  for (int b0 = 0; b0 < HB_BINS; b0 += 8) {
    unsigned c[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = __hip_atomic_load(hq + b0 + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      cum += c[j];
      if (cum >= (unsigned)kq) return hb_edge(base, b0 + j);
    }
  }
  return INFINITY;
}

constexpr int V2_ROWS = 32;  // gallery rows per tile
// tiles between two exchanges of the shared per-query bound (power of two; env
// ARTSBIR_KNN_KB=0 turns the exchange off in the one-call path)
#ifndef KB_SYNC_TILES
#define KB_SYNC_TILES 128  // round 5, after the prefetch fix: 32 / 64 / 128 -> 11.44 / 11.20 / 11.14 ms (profiles/r5_knn_kb.txt)
#endif
constexpr int KB_SYNC = KB_SYNC_TILES;
constexpr int V2_WAVES = 8;  // 8 x 32 = 256 queries per workgroup

template <int KB>
struct V2 {
  static constexpr int RB = 32 * KB + 16;               // augmented row bytes (Dp bf16 + 16)
  static constexpr int SLOTS = V2_ROWS * RB / 16;       // 16-B slots per tile
  static constexpr int NI = (SLOTS + 63) / 64;          // DMA instructions per tile
  static constexpr int STAGE = NI * 1024;
  // KNN_NST 4: three tiles in flight instead of two; the LDS it takes comes
  // from the slow path's staging, which then holds half a wave's rows per pass.
  // Measured slower again once the per-tile drain was gone (scan 11.2 -> 12.0 ms,
  // profiles/r5_knn_nst4.txt; round 4's 4-stage build ran under that drain), so
  // the DMA ring's depth does not bound the scan: 3 stays
#ifndef KNN_NST
#define KNN_NST 3
#endif
  static constexpr int NST = KNN_NST;
  static constexpr int SROWS = NST == 4 ? 16 : 32;       // staged rows per slow-path pass
  static constexpr int SP = 33;                          // staging pitch (floats)
  static constexpr int WSTG = SROWS * SP + (SROWS == 32 ? 0 : 32);  // + the 32 columns' |g|^2 (in the row padding at 32 rows)
  static constexpr int STG = V2_WAVES * WSTG * 4;
  static constexpr int ROWS = V2_WAVES * 32;
  static constexpr int LDS = NST * STAGE + STG + 5 * ROWS * 4;
  static_assert(LDS <= 163840, "LDS");
  static_assert((NI + V2_WAVES - 1) / V2_WAVES <= 5, "rvm_wait_n covers at most 5 DMA per wave");
  static_assert((NI + V2_WAVES / 2 - 1) / (V2_WAVES / 2) <= 10, "rvm_wait_n covers at most 10 DMA per wave");
};

// scan statistics (diagnostics, ARTSBIR_KNN_STAT=1): wave-tiles, slow-path
// entries, list insertions (summed per wave, one atomic per wave at the end)
// and the exact merge's live candidates (summed over queries)
__device__ unsigned long long g_knn_stat[4];
static bool knn_stat_on() {
  static const bool on = [] { const char* e = getenv("ARTSBIR_KNN_STAT"); return e && atoi(e) != 0; }();
  return on;
}

// QH: query halves per wave.  1: 8 waves of 32 queries (two waves per SIMD);
// 2: 4 waves of 64 (one wave per SIMD, the A fragments of both halves resident:
// 2 KB registers per lane at D = 512, AGPRs included), so each B fragment read
// from LDS feeds two MFMAs — half the LDS reads per MAC — and every lane owns a
// query row in the list / slow path (ARTSBIR_KNN_QH, knn_qh())
template <int KB, int QH = 1>
__global__ void __launch_bounds__(64 * V2_WAVES / QH, 1) knn_scan_v2_kernel(KnnScanArgs a, int stat) {
  using C = V2<KB>;
  constexpr int NWV = V2_WAVES / QH;  // waves of the workgroup
  static_assert(QH == 1 || (QH == 2 && C::SROWS == 32), "QH 2: the 3-stage ring (full-tile staging)");
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];
  float* s_stage = reinterpret_cast<float*>(smem + C::NST * C::STAGE);
  float* s_thr = s_stage + V2_WAVES * C::WSTG;     // [256] 16th smallest so far (-INF: row unused)
  float* s_crit = s_thr + C::ROWS;                 // [256] max(thr, band hi)
  float* s_lo = s_crit + C::ROWS;                  // [256] rank band (hi < 0: no band)
  float* s_hi = s_lo + C::ROWS;
  float* s_qsq = s_hi + C::ROWS;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntq = (a.Nq + C::ROWS - 1) / C::ROWS;
  int lid = (int)blockIdx.x;
  {  // the query tiles of one gallery chunk on one XCD at the same time (shared L2)
    const int nwg = (int)gridDim.x;
    if (nwg >= 8) {
      const int q8 = nwg / 8, r8 = nwg % 8, x = lid % 8;
      lid = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + lid / 8;
    }
  }
  const int chunk = lid / ntq, qt = lid % ntq;
  const int qb = qt * C::ROWS;
  const int rows_per_chunk = a.tiles_per_chunk * 128;
  const int g0 = chunk * rows_per_chunk;
  const int nrows = min(a.Ng - g0, rows_per_chunk);
  if (nrows <= 0) return;
  const int ntiles = (nrows + V2_ROWS - 1) / V2_ROWS;

  const __amdgpu_buffer_rsrc_t gr =
      rrsrc(reinterpret_cast<const char*>(a.g) + (long long)g0 * C::RB, (long long)(a.Ng - g0) * C::RB);
  // a tile is NI (33 at D = 512) 1-KB pieces over 8 waves: the wave issuing
  // the odd piece rotates with the tile (KNN_ROT), so no wave is the one every
  // barrier waits for
#ifndef KNN_ROT
#define KNN_ROT 1
#endif
  auto w_of = [&](int t) { return KNN_ROT ? (wid + t) & (NWV - 1) : wid; };
  auto ni_of = [&](int t) { const int w2 = w_of(t); return w2 < C::NI ? (C::NI - w2 + NWV - 1) / NWV : 0; };
  auto issue_tile = [&](int t) {
    char* st = smem + (t % C::NST) * C::STAGE;
    const unsigned gb = (unsigned)(t * V2_ROWS * C::RB);
    for (int i = w_of(t); i < C::NI; i += NWV) rdma16(gr, st + i * 1024, gb + (unsigned)((i * 64 + lane) * 16));
  };
  issue_tile(0);
  if (ntiles > 1) issue_tile(1);
  if (C::NST == 4 && ntiles > 2) issue_tile(2);

  const float* band_lo = a.lo;
  const float* band_hi = a.hi;
  if (tid < C::ROWS) {
    const int q = qb + tid;
    const bool ok = q < a.Nq;
    float t0 = (ok && a.thr0) ? a.thr0[q] : INFINITY;
    if (ok && a.kb) t0 = fminf(t0, kb_bound(a.kb[q], a.rel * sqrtf(a.qsq[q] * (a.gsq_max_p ? *a.gsq_max_p : a.gsq_max)) * 1.001f + 1e-3f));
    s_thr[tid] = ok ? t0 : -INFINITY;
    s_lo[tid] = (band_lo && ok) ? band_lo[q] : -1.f;
    s_hi[tid] = (band_lo && ok) ? band_hi[q] : -1.f;
    s_qsq[tid] = ok ? a.qsq[q] : 0.f;
    s_crit[tid] = ok ? fmaxf(t0, s_hi[tid]) : -INFINITY;
  }
  const int r32 = lane & 31, h = lane >> 5;
  const __amdgpu_buffer_rsrc_t qr = rrsrc(reinterpret_cast<const bf16*>(a.q) + (long long)qb * (16 * KB),
                                          (long long)(a.Nq - qb) * (32 * KB));
  uint4 af[QH][KB];
#pragma unroll
  for (int qh = 0; qh < QH; ++qh)
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
      af[qh][kb] = rload(qr, (unsigned)(((wid * 32 * QH + qh * 32 + r32) * 16 * KB + kb * 16 + 8 * h) * 2));
  // owner state: lane r < 32 owns row r of the wave (QH 2: lane l owns row l,
  // half l >> 5), with its e and accumulator half in the 32x32 accumulator
  const bool owner = QH == 2 || lane < 32;
  const int ohalf = QH == 2 ? lane >> 5 : 0;
  const int orow = lane & 31;
  const int oe = (orow & 3) + 4 * (orow >> 3), oh = (orow >> 2) & 1;
  const int R_own = wid * 32 * QH + ohalf * 32 + orow;
  float lst_d[KT];
  int lst_i[KT];
#pragma unroll
  for (int i = 0; i < KT; ++i) { lst_d[i] = INFINITY; lst_i[i] = -1; }
  int mycnt = 0;
  rvm_wait<0>();
  // the A fragments are resident from here on: launder them through an empty asm
  // so that the compiler's vmcnt tracking does not wait on (our hand-counted
  // DMAs behind) their loads inside the tile loop
#pragma unroll
  for (int qh = 0; qh < QH; ++qh)
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
      asm volatile("" : "+v"(af[qh][kb].x), "+v"(af[qh][kb].y), "+v"(af[qh][kb].z), "+v"(af[qh][kb].w));
  __syncthreads();
  // prefilter: t = |g|^2 - 2 q.g <= crit - |q|^2 + slack, a superset of
  // d2 = (|q|^2 + |g|^2) - 2 q.g <= crit whatever the rounding of either form
  // (every magnitude is <= 2 (|q|^2 + gsq_max), each rounding <= 2^-24 of it)
  const float gmax = a.gsq_max_p ? *a.gsq_max_p : a.gsq_max;
  float critp[QH][16];
  auto load_crit = [&]() {
#pragma unroll
    for (int qh = 0; qh < QH; ++qh)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int R = wid * 32 * QH + qh * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        const float qs = s_qsq[R];
        critp[qh][e] = (s_crit[R] - qs) + 0x1p-18f * (qs + gmax);
      }
  };
  load_crit();
  float* stg0 = s_stage + wid * QH * C::WSTG;  // half qh's staging at stg0 + qh * WSTG
  float* sg = stg0 + (C::SROWS == 32 ? 32 : C::SROWS * C::SP);  // column c's |g|^2 at sg[c * gstr]
  constexpr int gstr = C::SROWS == 32 ? C::SP : 1;
  const int q_own = qb + R_own;
  const float eps_own = q_own < a.Nq ? a.rel * sqrtf(a.qsq[q_own] * gmax) * 1.001f + 1e-3f : 0.f;
  float thr_g = s_thr[R_own];  // best shared bound seen (with thr0)
  int pub_wm = g0;              // list items with a gallery index >= pub_wm are not yet in the histogram
  unsigned hbq = 0;             // the query's histogram base key (0: not known yet)

  bool atom = false;  // this wave issued a global atomic since its last DMA wait
  unsigned st_entries = 0, st_ins = 0;
  for (int t = 0; t < ntiles; ++t) {
    if (t + C::NST - 1 < ntiles) issue_tile(t + C::NST - 1);
    const char* st = smem + (t % C::NST) * C::STAGE;
    const char* bp = st + r32 * C::RB + h * 16;
    // B fragments PF reads ahead of their MFMA, pinned in that order (left
    // alone, the scheduler either hoists all KB reads and runs out of registers
    // or issues each read just one MFMA before its use and exposes the LDS latency)
    // (KNN_PF: at 6 the kernel needs 256 VGPRs plus a 16-B spill whose reload
    // before the first MFMA of every tile carried s_waitcnt vmcnt(0), draining
    // the DMA ring each tile; 4 spills nothing)
#ifndef KNN_PF
#define KNN_PF 4
#endif
    constexpr int PF = KB < KNN_PF ? KB : KNN_PF;
    f32x16 acc[QH];
#pragma unroll
    for (int qh = 0; qh < QH; ++qh) acc[qh] = f32x16{};
    uint4 bq[KB];
#ifndef KNN_ABL
#define KNN_ABL 0  // timing ablations of a diagnostic build only (1: no list work, 2: no MFMAs; tools/gpu/r4_knn_abl.sh)
#endif
#pragma unroll
    for (int j = 0; j < PF; ++j) bq[j] = *reinterpret_cast<const uint4*>(bp + j * 32);
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      if (kb + PF < KB) bq[kb + PF] = *reinterpret_cast<const uint4*>(bp + (kb + PF) * 32);
#pragma unroll
      for (int qh = 0; qh < QH; ++qh) {
        if (KNN_ABL & 2)
          acc[qh][kb & 15] += __uint_as_float(bq[kb].x & 0x80000000u);
        else if (QH == 2) {
          // the A fragments stay in AGPRs (the MFMA reads them there; the builtin
          // had the compiler copy each one to VGPRs first: 244 v_accvgpr_read
          // per tile); acc in VGPRs for the prefilter
          typedef unsigned kv_u4 __attribute__((ext_vector_type(4)));
          const kv_u4 av = __builtin_bit_cast(kv_u4, af[qh][kb]), bv = __builtin_bit_cast(kv_u4, bq[kb]);
          if (kb == 0)
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=v"(acc[qh]) : "a"(av), "v"(bv));
          else
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc[qh]) : "a"(av), "v"(bv));
        } else
          acc[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(&af[qh][kb]),
                                                            *reinterpret_cast<const bf16x8*>(&bq[kb]), acc[qh], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // the hand-issued MFMAs' results are read by vector instructions next: the
    // 16-pass XDL write -> VALU read hazard (18 wait states) the compiler cannot see
    if (QH == 2 && !(KNN_ABL & 2)) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
    const int bn = g0 + t * V2_ROWS;
    const bool cvalid = bn + r32 < a.Ng;
    const float gsq = cvalid ? *reinterpret_cast<const float*>(st + r32 * C::RB + 32 * KB) : INFINITY;
    // stage t+1 landed (this wave's DMAs; the barrier publishes everyone's).  The
    // barrier sits BEFORE this tile's epilogue: a wave busy inserting list hits
    // then overlaps the next tile's MFMAs of the other waves instead of holding
    // them at the barrier.  So after it, stage t may already be refilled (DMA of
    // tile t+3): the epilogue reads no stage, only gsq (saved above) and its own
    // wave's LDS.  An atomic of the previous epilogue forces the full wait.
    if (t + 1 < ntiles) {
      if (t + 2 < ntiles && !__builtin_amdgcn_ballot_w64(atom)) {
        if (C::NST == 4 && t + 3 < ntiles)
          rvm_wait_n(ni_of(t + 2) + ni_of(t + 3));
        else
          rvm_wait_n(ni_of(t + 2));
      } else {
        rvm_wait<0>();
      }
    }
    atom = false;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of stage t (gsq) are done
    __syncthreads();
    bool any = false;
#pragma unroll
    for (int qh = 0; qh < QH; ++qh)
#pragma unroll
      for (int e = 0; e < 16; ++e) any |= fmaf(-2.f, acc[qh][e], gsq) <= critp[qh][e];
    if (KNN_ABL & 1) {
      st_entries += __builtin_amdgcn_ballot_w64(any) ? 1u : 0u;
      any = false;
    }
    if (__builtin_amdgcn_ballot_w64(any)) {
      ++st_entries;
      // stage the raw dot products of every row with a prefilter hit; the owner
      // of each row re-evaluates its hits exactly (d2 with the same formula as
      // knn_scan_kernel): list insertion, certainly-closer count, uncertain queue
      unsigned mymask = 0;
      if (lane < 32) sg[r32 * gstr] = gsq;  // column r32's |g|^2 (INF past Ng)
#pragma unroll
      for (int qh = 0; qh < QH; ++qh) {
        float* stg = stg0 + qh * C::WSTG;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const unsigned long long m = __builtin_amdgcn_ballot_w64(fmaf(-2.f, acc[qh][e], gsq) <= critp[qh][e]);
          if (m) {
            if (C::SROWS == 32) stg[((e & 3) + 8 * (e >> 2) + 4 * h) * C::SP + r32] = acc[qh][e];
            if (oe == e && ohalf == qh) mymask = oh ? (unsigned)(m >> 32) : (unsigned)m;
          }
        }
      }
      float* stg = stg0 + ohalf * C::WSTG;  // the owner's half
      bool changed = false;
      // every lane reads its (owner) row's state: lanes >= 32 mirror row lane - 32
      const float qs = s_qsq[R_own], hi = s_hi[R_own];
      float thr = s_thr[R_own];
      // SROWS 16: two passes, the rows of lane half hp (h == hp) staged at
      // (e & 3) + 4 (e >> 2), their owners (oh == hp) evaluating in between
#pragma unroll
      for (int hp = 0; hp < (C::SROWS == 32 ? 1 : 2); ++hp) {
      if (C::SROWS == 16) {
        if (hp) {  // pass 0's owners are done with the staging
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
          __builtin_amdgcn_wave_barrier();
        }
        if (h == hp) {
#pragma unroll
          for (int e = 0; e < 16; ++e) stg[((e & 3) + 4 * (e >> 2)) * C::SP + r32] = acc[0][e];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (owner && mymask && (C::SROWS == 32 || oh == hp)) {
        const float lo = s_lo[R_own];
        const float* srow = stg + (C::SROWS == 32 ? orow : oe) * C::SP;
        while (mymask) {
          const int c = __builtin_ctz(mymask);
          mymask &= mymask - 1;
          const bool valid = bn + c < a.Ng;
          const float g2 = sg[c * gstr];
          const float d2 = fmaf(-2.f, srow[c], qs + g2);
          if (d2 < thr) {
            ++st_ins;
            float x = d2;
            int xi = bn + c;
            // compare-swap down the sorted list.  Items reach a chunk's list in
            // increasing gallery index (tiles in order, columns in ctz order), so
            // a listed item equal in value always has the lower index and stays
            // ahead: the strict compare alone keeps the (value, index) order
#pragma unroll
            for (int i = 0; i < KT; ++i) {
              const bool sw = x < lst_d[i];
              const float td = lst_d[i];
              const int ti = lst_i[i];
              lst_d[i] = sw ? x : td;
              lst_i[i] = sw ? xi : ti;
              x = sw ? td : x;
              xi = sw ? ti : xi;
            }
            thr = fminf(lst_d[KT - 1], thr_g);
            changed = true;
          }
          if (hi >= 0.f && valid) {
            if (d2 < lo) {
              ++mycnt;
            } else if (d2 <= hi) {
              const int k = atomicAdd(a.unc + 2 * a.unc_cap, 1);
              if (k < a.unc_cap) { a.unc[2 * k] = qb + R_own; a.unc[2 * k + 1] = bn + c; }
              atom = true;
            }
          }
        }
        if (changed) {
          s_thr[R_own] = thr;
          s_crit[R_own] = fmaxf(thr, hi);
        }
      }
      }
      if (__builtin_amdgcn_ballot_w64(changed)) {
        // refresh the prefilter bounds from the owner lanes' registers (readlane:
        // no fence, no LDS round trip); the same value load_crit() would read
        // (padding rows q >= Nq keep -INF, as load_crit() reads them)
        const float mine = q_own < a.Nq ? (fmaxf(thr, hi) - qs) + 0x1p-18f * (qs + gmax) : -INFINITY;
#pragma unroll
        for (int qh = 0; qh < QH; ++qh)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int r0 = qh * 32 + (e & 3) + 8 * (e >> 2);
            const float n0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mine), r0));
            const float n1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mine), r0 + 4));
            critp[qh][e] = h ? n1 : n0;
          }
      }
    }
    if (a.kb && (((t & (KB_SYNC - 1)) == KB_SYNC - 1) || t + 1 == ntiles)) {
      // every KB_SYNC tiles and once more at the chunk's end (a chunk of at most
      // KB_SYNC tiles, and the ragged last one, still publish what they found),
      // the query's bound shared by every chunk (one
      // returning atomicMin per row): publish this chunk's kq-th smallest so far
      // and take the best any chunk has published.  The pipeline drains here
      // once (the atomic's value is used at once), instead of at every list
      // change: the chunks running beside this one, and those that ran before
      // it, then cut its slow-path entries to the items that can still reach
      // the global top k (kb_bound above).
      rvm_wait<0>();
      bool upd = false, pub = false;
      if (owner && q_own < a.Nq) {
        float kth = INFINITY;
#pragma unroll
        for (int i = 0; i < KT; ++i) kth = (i == a.kq - 1 && lst_i[i] >= 0) ? lst_d[i] : kth;
        float bnd = kth;
        if (a.hist) {
          if (!hbq) {
            if (kth < INFINITY) {
              const unsigned want = max(hb_key(kth + 2.f * eps_own), (unsigned)HB_BINS) - (HB_BINS - 1);
              const unsigned old = atomicCAS(a.hbase + q_own, 0u, want);
              hbq = old ? old : want;
            } else {
              hbq = __hip_atomic_load(a.hbase + q_own, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
          if (hbq) {
            unsigned* hq = a.hist + (long long)q_own * HB_BINS;
#pragma unroll
            for (int i = 0; i < KT; ++i) {
              if (lst_i[i] >= pub_wm) {
                const int b = hb_bin(lst_d[i], hbq);
                if (b < HB_BINS) {
                  atomicAdd(hq + b, 1u);
                  pub = true;
                }
              }
            }
            pub_wm = g0 + (t + 1) * V2_ROWS;
            if (pub) bnd = fminf(bnd, hb_bound(hq, hbq, a.kq));
          }
        }
        const unsigned mine = kb_enc(bnd);
        const unsigned old = atomicMin(a.kb + q_own, mine);
        const float g = kb_bound(old < mine ? old : mine, eps_own);
        if (g < thr_g) {
          thr_g = g;
          const float cur = s_thr[R_own];
          if (g < cur) {
            s_thr[R_own] = g;
            s_crit[R_own] = fmaxf(g, s_hi[R_own]);
            upd = true;
          }
        }
      }
      // drained above; the returning atomics were waited for at their use, the
      // histogram adds were not: they force the next tile's full wait
      atom = pub;
      if (__builtin_amdgcn_ballot_w64(upd)) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        load_crit();
      }
    }
  }
  if (stat) {
    unsigned ins = st_ins;
    for (int off = 32; off; off >>= 1) ins += __shfl_xor(ins, off, 64);
    if (lane == 0) {
      atomicAdd(&g_knn_stat[0], (unsigned long long)ntiles);
      atomicAdd(&g_knn_stat[1], (unsigned long long)st_entries);
      atomicAdd(&g_knn_stat[2], (unsigned long long)ins);
    }
  }
  if (owner) {
    const int q = qb + R_own;
    if (q < a.Nq) {
      if (mycnt) atomicAdd(a.cnt + q, mycnt);
      const long long o = ((long long)q * a.nchunks + chunk) * KT;
#pragma unroll
      for (int i = 0; i < KT; ++i) {
        a.cand_d[o + i] = lst_d[i];
        a.cand_i[o + i] = lst_i[i];
      }
    }
  }
}

// queries per wave of the v2 scan: ARTSBIR_KNN_QH=2 (64, one wave per SIMD) or 1 (32)
static int knn_qh() {
  static const int qh = [] { const char* e = getenv("ARTSBIR_KNN_QH"); return e && atoi(e) == 2 ? 2 : 1; }();
  return qh;
}

static void knn_scan_v2_launch(int Dp, unsigned grid, const KnnScanArgs& a, int stat, hipStream_t st) {
  const dim3 g(grid);
  if (knn_qh() == 2 && Dp == 512) {  // the register budget of two halves is sized for D = 512
    hipLaunchKernelGGL((knn_scan_v2_kernel<32, 2>), g, dim3(256), 0, st, a, stat);
    return;
  }
  switch (Dp) {
    case 64: hipLaunchKernelGGL((knn_scan_v2_kernel<4, 1>), g, dim3(512), 0, st, a, stat); break;
    case 128: hipLaunchKernelGGL((knn_scan_v2_kernel<8, 1>), g, dim3(512), 0, st, a, stat); break;
    case 256: hipLaunchKernelGGL((knn_scan_v2_kernel<16, 1>), g, dim3(512), 0, st, a, stat); break;
    default: hipLaunchKernelGGL((knn_scan_v2_kernel<32, 1>), g, dim3(512), 0, st, a, stat); break;
  }
}

// augmented bf16 rows for knn_scan_v2: [n][Dp + 8], columns Dp..Dp+1 = f32 |x|^2
// (normalize: unit rows for the cosine metric, as rows_prep_kernel)
__global__ void rows_prep_aug_kernel(const float* __restrict__ x, int n, int D, int Dp, float* __restrict__ sq,
                                     bf16* __restrict__ xa, int normalize) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (row >= n) return;
  const float* r = x + (long long)row * D;
  const float sc = row_scale(r, D, lane, normalize);
  bf16* o = xa + (long long)row * (Dp + 8);
  float s = 0.f;
  if (row_vec_ok(r, D)) {
    // 8 consecutive columns per lane: two 16-B loads, one 16-B store of the
    // bf16 copy (the row pitch 2 (Dp + 8) B is a multiple of 16)
    for (int d0 = lane * 8; d0 < Dp; d0 += 512) {
      float v[8];
      row_load8(r, D, d0, sc, v);
      bf16 h[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s = fmaf(v[j], v[j], s);  // explicit fma: the same rounding in both kernels
        h[j] = (bf16)v[j];
      }
      *reinterpret_cast<uint4*>(o + d0) = *reinterpret_cast<const uint4*>(h);
    }
  } else {
    for (int d = lane; d < Dp; d += 64) {
      const float v = d < D ? r[d] * sc : 0.f;
      s = fmaf(v, v, s);
      o[d] = (bf16)v;
    }
  }
  s = warp_sum(s);
  if (lane < 8) {
    const unsigned bits = __float_as_uint(s);
    unsigned short v = 0;
    if (lane == 0) v = (unsigned short)(bits & 0xffffu);
    if (lane == 1) v = (unsigned short)(bits >> 16);
    reinterpret_cast<unsigned short*>(o)[Dp + lane] = v;
  }
  if (lane == 0) sq[row] = s;
}

// ------------------------------------------------------------ exact merge
// one workgroup per query: exact f64 distances of every candidate, top-k by
// (distance, global index), verification of the chunk lists.
__global__ void __launch_bounds__(256) knn_merge_kernel(const float* __restrict__ q, const float* __restrict__ g, int D,
                                                        int nchunks, const float* __restrict__ cand_d,
                                                        const int* __restrict__ cand_i, const float* __restrict__ qsq,
                                                        float gsq_max, float rel, long long g_base, int k,
                                                        long long* __restrict__ out_i, double* __restrict__ out_d,
                                                        int* __restrict__ flag, int metric,
                                                        const float* __restrict__ qeps, long long n_g) {
  extern __shared__ char sm[];
  const int nc = nchunks * KT;
  double* ed = reinterpret_cast<double*>(sm);           // [nc]
  int* ei = reinterpret_cast<int*>(ed + nc);            // [nc]
  const int qi = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const float* qr = q + (long long)qi * D;
  const float* cd = cand_d + (long long)qi * nc;
  const int* ci = cand_i + (long long)qi * nc;
  const double eps = qeps ? (double)qeps[qi] : rel * sqrt((double)qsq[qi] * gsq_max) + 1e-3;
  __shared__ double rd[4];
  __shared__ int ri[4], rslot[4];
  // (1) a_k = k-th smallest approximate value: the k items with approx <= a_k have
  //     exact d^2 <= a_k + eps, so every true top-k item has approx <= a_k + 2 eps
  for (int c = threadIdx.x; c < nc; c += blockDim.x) { ed[c] = ci[c] >= 0 ? (double)cd[c] : INFINITY; ei[c] = c; }
  __syncthreads();
  double ak = INFINITY;
  for (int r = 0; r < k; ++r) {
    double bd = INFINITY;
    int bs = -1;
    for (int c = threadIdx.x; c < nc; c += blockDim.x)
      if (ei[c] >= 0 && ed[c] < bd) { bd = ed[c]; bs = c; }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double od = __shfl_xor(bd, o, 64);
      const int os = __shfl_xor(bs, o, 64);
      if (od < bd) { bd = od; bs = os; }
    }
    if (lane == 0) { rd[wid] = bd; rslot[wid] = bs; }
    __syncthreads();
    if (threadIdx.x == 0) {
      double b = rd[0];
      int s2 = rslot[0];
      for (int w = 1; w < (int)blockDim.x / 64; ++w)
        if (rd[w] < b) { b = rd[w]; s2 = rslot[w]; }
      if (s2 >= 0) ei[s2] = -1;
      rd[0] = b;
    }
    __syncthreads();
    ak = rd[0];
    __syncthreads();
  }
  const double cut = ak + 2.0 * eps;
  // (2) exact f64 distances only for candidates that can still be in the top-k
  for (int c = wid; c < nc; c += blockDim.x / 64) {
    const int gi = ci[c];
    double d = INFINITY;
    const bool live = gi >= 0 && (double)cd[c] <= cut;
    if (live) d = exact_key(qr, g + (long long)gi * D, D, lane, metric);
    if (lane == 0) { ed[c] = d; ei[c] = live ? gi : -1; }
  }
  __syncthreads();
  // (3) k rounds of a block-wide argmin on (exact distance, index)
  double kth = INFINITY;
  for (int r = 0; r < k; ++r) {
    double bd = INFINITY;
    int bi = 0x7fffffff, bs = -1;
    for (int c = threadIdx.x; c < nc; c += blockDim.x) {
      const double d = ed[c];
      const int i = ei[c];
      if (i >= 0 && (d < bd || (d == bd && i < bi))) { bd = d; bi = i; bs = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double od = __shfl_xor(bd, o, 64);
      const int oi = __shfl_xor(bi, o, 64), os = __shfl_xor(bs, o, 64);
      if (od < bd || (od == bd && oi < bi)) { bd = od; bi = oi; bs = os; }
    }
    if (lane == 0) { rd[wid] = bd; ri[wid] = bi; rslot[wid] = bs; }
    __syncthreads();
    if (threadIdx.x == 0) {
      double b = rd[0];
      int bi2 = ri[0], bs2 = rslot[0];
      for (int w = 1; w < (int)blockDim.x / 64; ++w)
        if (rd[w] < b || (rd[w] == b && ri[w] < bi2)) { b = rd[w]; bi2 = ri[w]; bs2 = rslot[w]; }
      out_i[(long long)qi * k + r] = bs2 >= 0 ? g_base + bi2 : -1;
      out_d[(long long)qi * k + r] = b;
      if (bs2 >= 0) ei[bs2] = -1;  // remove
      rd[0] = b;
    }
    __syncthreads();
    kth = rd[0];
    __syncthreads();
  }
  // verification: a full chunk list whose last approximate value is within the
  // error band of the k-th exact distance may have dropped a true top-k item
  // (also when the chunk lists hold fewer than min(k, n_g) items at all)
  if (threadIdx.x == 0) {
    int bad = 0;
    long long valid = 0;
    for (int c = 0; c < nchunks; ++c) {
      const float last = cd[c * KT + KT - 1];
      if (ci[c * KT + KT - 1] >= 0 && (double)last - eps <= key_d2(kth, metric)) bad = 1;
      for (int i = 0; i < KT; ++i) valid += ci[c * KT + i] >= 0;
    }
    if (n_g > 0 && valid < (n_g < k ? n_g : (long long)k)) bad = 1;
    flag[qi] = bad;
  }
}

// The same merge with one wave per query and no workgroup barriers (the block
// version above spends most of its time in k rounds of block-wide argmin
// behind __syncthreads): the candidates of a query sit in registers, NPL per
// lane (nc <= 64 NPL); a_k by bisection over their order-preserving u32 keys;
// the live candidates compacted into LDS by ballot; their exact keys four at a
// time (more gathers in flight per wave; each key summed in exactly the order
// of exact_key, so results are bit-identical); k rounds of wave argmin on
// (exact key, index).  Outputs, flag and semantics as knn_merge_kernel.
__device__ __forceinline__ void exact_keys4(const float* q, const float* const* gr, int n, int D, int lane, int metric,
                                            double* out) {
  double s0[4] = {0.0, 0.0, 0.0, 0.0}, s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  for (int d = lane; d < D; d += 64) {
    const double a = q[d];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (u < n) {
        const double b = gr[u][d];
        if (metric == 0) {
          const double t = (a - b) + 1e-6;
          s0[u] += t * t;
        } else {
          s0[u] += a * b;
          s1[u] += a * a;
          s2[u] += b * b;
        }
      }
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s0[u] += __shfl_xor(s0[u], o, 64);
      if (metric) {
        s1[u] += __shfl_xor(s1[u], o, 64);
        s2[u] += __shfl_xor(s2[u], o, 64);
      }
    }
    out[u] = metric == 0 ? sqrt(s0[u]) : 1.0 - s0[u] / (fmax(sqrt(s1[u]), 1e-8) * fmax(sqrt(s2[u]), 1e-8));
  }
}

// the same keys with the whole rows loaded first (D <= 64 NI): every gather of a
// pass is in flight at once instead of one column block per round trip; the
// per-lane sums still run over d = lane, lane + 64, ... in order, so the keys
// are bit-identical to exact_key's
template <int NI>
__device__ __forceinline__ void exact_keys4_reg(const float* qreg, const float* const* gr, int n, int D, int lane,
                                                int metric, double* out) {
  // unconditional loads (clamped column; rows u >= n repeat row 0) so that all
  // 4 NI gathers are in flight together: a predicated load compiles to a branch
  // with a wait at its join, one round trip per load
  float gv[4][NI];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int i = 0; i < NI; ++i) gv[u][i] = gr[u][min(lane + 64 * i, D - 1)];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if (lane + 64 * i < D) {
        const double a = qreg[i], b = gv[u][i];
        if (metric == 0) {
          const double t = (a - b) + 1e-6;
          s0 += t * t;
        } else {
          s0 += a * b;
          s1 += a * a;
          s2 += b * b;
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s0 += __shfl_xor(s0, o, 64);
      if (metric) {
        s1 += __shfl_xor(s1, o, 64);
        s2 += __shfl_xor(s2, o, 64);
      }
    }
    out[u] = metric == 0 ? sqrt(s0) : 1.0 - s0 / (fmax(sqrt(s1), 1e-8) * fmax(sqrt(s2), 1e-8));
  }
}

template <int NPL>
__global__ void __launch_bounds__(64) knn_merge_wave_kernel(const float* __restrict__ q, const float* __restrict__ g,
                                                            int D, int nchunks, const float* __restrict__ cand_d,
                                                            const int* __restrict__ cand_i,
                                                            const float* __restrict__ qsq, float gsq_max, float rel,
                                                            long long g_base, int k, long long* __restrict__ out_i,
                                                            double* __restrict__ out_d, int* __restrict__ flag,
                                                            int metric, const float* __restrict__ qeps, long long n_g,
                                                            int stat) {
  extern __shared__ char sm[];
  const int nc = nchunks * KT;
  double* ed = reinterpret_cast<double*>(sm);  // [nc] exact keys of the live candidates (compacted)
  int* ei = reinterpret_cast<int*>(ed + nc);   // [nc] their gallery indices (-1: taken)
  const int qi = blockIdx.x, lane = threadIdx.x;
  const float* qr = q + (long long)qi * D;
  const float* cd = cand_d + (long long)qi * nc;
  const int* ci = cand_i + (long long)qi * nc;
  const double eps = qeps ? (double)qeps[qi] : rel * sqrt((double)qsq[qi] * gsq_max) + 1e-3;
  float av[NPL];
  int ai[NPL];
  unsigned nvalid = 0;
#pragma unroll
  for (int j = 0; j < NPL; ++j) {  // unconditional (clamped) loads, masked after
    const int c = min(lane + 64 * j, nc - 1);
    ai[j] = ci[c];
    av[j] = cd[c];
  }
#pragma unroll
  for (int j = 0; j < NPL; ++j) {
    if (lane + 64 * j >= nc) ai[j] = -1;
    if (ai[j] < 0) av[j] = INFINITY;
    nvalid += (unsigned)__popcll(__builtin_amdgcn_ballot_w64(ai[j] >= 0));
  }
  // (1) a_k, the k-th smallest approximate value (as knn_merge_kernel step 1)
  double ak = INFINITY;
  if (nvalid >= (unsigned)k) {
    unsigned lo = 0u, hi = 0xffffffffu;
    while (lo < hi) {
      const unsigned mid = lo + ((hi - lo) >> 1);
      unsigned cnt = 0;
#pragma unroll
      for (int j = 0; j < NPL; ++j)
        cnt += (unsigned)__popcll(__builtin_amdgcn_ballot_w64(ai[j] >= 0 && kb_enc(av[j]) <= mid));
      if (cnt >= (unsigned)k) hi = mid; else lo = mid + 1;
    }
    ak = (double)kb_dec(lo);
  }
  const double cut = ak + 2.0 * eps;
  // (2) compact the live candidates
  int L = 0;
#pragma unroll
  for (int j = 0; j < NPL; ++j) {
    const bool live = ai[j] >= 0 && (double)av[j] <= cut;
    const unsigned long long m = __builtin_amdgcn_ballot_w64(live);
    if (live) {
      const int pos = L + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
      ei[pos] = ai[j];
    }
    L += (int)__popcll(m);
  }
  if (stat && lane == 0) atomicAdd(&g_knn_stat[3], (unsigned long long)L);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // (3) exact keys, four candidates per pass
  constexpr int NI = 8;  // rows of up to 512 columns held in registers
  float qreg[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) qreg[i] = qr[min(lane + 64 * i, D - 1)];  // columns >= D are never summed
  for (int j0 = 0; j0 < L; j0 += 4) {
    const int n = min(4, L - j0);
    const float* gr[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) gr[u] = g + (long long)ei[j0 + (u < n ? u : 0)] * D;
    double kk[4];
    if (D <= 64 * NI)
      exact_keys4_reg<NI>(qreg, gr, n, D, lane, metric, kk);
    else
      exact_keys4(qr, gr, n, D, lane, metric, kk);
    if (lane == 0) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (u < n) ed[j0 + u] = kk[u];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // (4) k rounds of wave argmin on (exact key, index)
  double kth = INFINITY;
  for (int r = 0; r < k; ++r) {
    double bd = INFINITY;
    int bi = 0x7fffffff, bs = -1;
    for (int j = lane; j < L; j += 64) {
      const int i = ei[j];
      const double d = ed[j];
      if (i >= 0 && (d < bd || (d == bd && i < bi))) { bd = d; bi = i; bs = j; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double od = __shfl_xor(bd, o, 64);
      const int oi = __shfl_xor(bi, o, 64), os = __shfl_xor(bs, o, 64);
      if (od < bd || (od == bd && oi < bi)) { bd = od; bi = oi; bs = os; }
    }
    if (lane == 0) {
      out_i[(long long)qi * k + r] = bs >= 0 ? g_base + bi : -1;
      out_d[(long long)qi * k + r] = bd;
      if (bs >= 0) ei[bs] = -1;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    kth = bd;
  }
  // (5) verification, as knn_merge_kernel
  int bad = 0;
  long long valid = 0;
  for (int c = lane; c < nchunks; c += 64) {
    const float last = cd[c * KT + KT - 1];
    if (ci[c * KT + KT - 1] >= 0 && (double)last - eps <= key_d2(kth, metric)) bad = 1;
  }
  valid = nvalid;
  bad = __builtin_amdgcn_ballot_w64(bad != 0) != 0;
  if (n_g > 0 && valid < (n_g < k ? n_g : (long long)k)) bad = 1;
  if (lane == 0) flag[qi] = bad;
}

// launches the one-wave merge when the candidates fit its registers (nc <= 1024)
static bool launch_merge_wave(int Q, hipStream_t st, const float* q, const float* g, int D, int nchunks,
                              const float* cand_d, const int* cand_i, const float* qsq, float gsq_max, float rel,
                              long long g_base, int k, long long* out_i, double* out_d, int* flag, int metric,
                              const float* qeps, long long n_g) {
  static const bool on = [] { const char* e = getenv("ARTSBIR_KNN_MERGE_WAVE"); return !e || atoi(e) != 0; }();
  const int nc = nchunks * KT;
  if (!on || nc > 1024) return false;
  const size_t sh = (size_t)nc * (sizeof(double) + sizeof(int));
#define ARTSBIR_MW(NPL)                                                                                            \
  hipLaunchKernelGGL(knn_merge_wave_kernel<NPL>, dim3(Q), dim3(64), sh, st, q, g, D, nchunks, cand_d, cand_i, qsq, \
                     gsq_max, rel, g_base, k, out_i, out_d, flag, metric, qeps, n_g, knn_stat_on() ? 1 : 0)
  if (nc <= 128) ARTSBIR_MW(2);
  else if (nc <= 256) ARTSBIR_MW(4);
  else if (nc <= 512) ARTSBIR_MW(8);
  else ARTSBIR_MW(16);
#undef ARTSBIR_MW
  return true;
}

// exact checks of the uncertain items of the rank count
__global__ void knn_uncertain_kernel(const float* __restrict__ q, const float* __restrict__ g, int D,
                                     const int* __restrict__ unc, int unc_cap, const double* __restrict__ dpos,
                                     const long long* __restrict__ pos, long long g_base, int* __restrict__ cnt,
                                     int metric) {
  const int lane = threadIdx.x & 63;
  const int n = min(unc[2 * unc_cap], unc_cap);
  for (int e = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); e < n; e += gridDim.x * (blockDim.x / 64)) {
    const int qi = unc[2 * e], gi = unc[2 * e + 1];
    const double d = exact_key(q + (long long)qi * D, g + (long long)gi * D, D, lane, metric);
    const double dp = dpos[qi];
    const long long ggi = g_base + gi;
    if (lane == 0 && (d < dp || (d == dp && ggi < pos[qi]))) atomicAdd(cnt + qi, 1);
  }
}

// exhaustive exact scan of one query (fallback for flagged queries, and the
// small-gallery path): writes all exact distances
__global__ void knn_exact_all_kernel(const float* __restrict__ q, const float* __restrict__ g, int D, int n,
                                     double* __restrict__ out, int metric) {
  const int lane = threadIdx.x & 63;
  for (int i = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); i < n; i += gridDim.x * (blockDim.x / 64)) {
    const double d = exact_key(q, g + (long long)i * D, D, lane, metric);
    if (lane == 0) out[i] = d;
  }
}

// nn.PairwiseDistance(p=2, eps=1e-6) with broadcasting of a one-row operand,
// f32 arithmetic as torch does it (utils.euclidean_distance)
__global__ void pairwise_l2_kernel(const float* __restrict__ x1, long long n1, const float* __restrict__ x2, long long n2,
                                   int D, float eps, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const long long n = n1 > n2 ? n1 : n2;
  for (long long i = blockIdx.x * (long long)(blockDim.x / 64) + (threadIdx.x >> 6); i < n;
       i += (long long)gridDim.x * (blockDim.x / 64)) {
    const float* a = x1 + (n1 == 1 ? 0 : i) * D;
    const float* b = x2 + (n2 == 1 ? 0 : i) * D;
    float s = 0.f;
    for (int d = lane; d < D; d += 64) {
      const float t = a[d] - b[d] + eps;
      s += t * t;
    }
    s = warp_sum(s);
    if (lane == 0) out[i] = sqrtf(s);
  }
}

// ------------------------------------------- one-call top-k (no host syncs)
// The kernels below complete artsbir_pairwise_l2_topk: every decision the
// multi-call protocol made on the host (max |g|^2, the uncertain-queue overflow,
// flagged queries) is made on the device.

// min and max of |g|^2 over the gallery into ext[0] (max), ext[1] (min) as f32
// bit patterns (non-negative floats order like their bits); ext preset to (0, +INF)
__global__ void sq_minmax_kernel(const float* __restrict__ sq, long long n, unsigned* __restrict__ ext) {
  float mx = 0.f, mn = INFINITY;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    mx = fmaxf(mx, sq[i]);
    mn = fminf(mn, sq[i]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    mn = fminf(mn, __shfl_xor(mn, o, 64));
  }
  // one atomic pair per workgroup (the atomics on two words serialise: one pair
  // per wave of a 1024-workgroup grid took ~95 us)
  __shared__ float smx[16], smn[16];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { smx[w] = mx; smn[w] = mn; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) { mx = fmaxf(mx, smx[i]); mn = fminf(mn, smn[i]); }
    atomicMax(ext, __float_as_uint(mx));
    atomicMin(ext + 1, __float_as_uint(mn));
  }
}

// per-query eps (query_eps) and the initial dpos (caller's value for shard
// calls, else -1); cnt and the uncertain-queue length start at 0
__global__ void knn_init_kernel(const float* __restrict__ qsq, const unsigned* __restrict__ ext, int nq, float rel,
                                int metric, const double* __restrict__ dpos_in, float* __restrict__ qeps,
                                double* __restrict__ dpos, int* __restrict__ cnt, int* __restrict__ unc_n) {
  const int qi = blockIdx.x * blockDim.x + threadIdx.x;
  if (qi == 0) *unc_n = 0;
  if (qi >= nq) return;
  const float gmax = __uint_as_float(ext[0]), gmin = __uint_as_float(ext[1]);
  qeps[qi] = (float)(query_eps(qsq[qi], gmax, gmin, rel, metric) * (1.0 + 1e-6));
  dpos[qi] = dpos_in ? dpos_in[qi] : -1.0;
  cnt[qi] = 0;
}

// uncertain-queue overflow (more uncertain items than unc_cap): recount every
// query's rank exhaustively in f64.  Both kernels return at once otherwise.
__global__ void knn_count_reset_kernel(const int* __restrict__ unc_n, int unc_cap, int nq, int* __restrict__ cnt) {
  if (*unc_n <= unc_cap) return;
  const int qi = blockIdx.x * blockDim.x + threadIdx.x;
  if (qi < nq) cnt[qi] = 0;
}

__global__ void __launch_bounds__(256) knn_count_exhaustive_kernel(const float* __restrict__ q,
                                                                   const float* __restrict__ g, int D, long long n,
                                                                   const int* __restrict__ unc_n, int unc_cap,
                                                                   const double* __restrict__ dpos,
                                                                   const long long* __restrict__ pos,
                                                                   long long g_base, int* __restrict__ cnt,
                                                                   int metric, int nq) {
  if (*unc_n <= unc_cap) return;  // the usual case: the grid is small so this costs ~nothing
  const int lane = threadIdx.x & 63;
  constexpr int SLICES = 64;  // workgroups per query
  for (long long job = blockIdx.x; job < (long long)nq * SLICES; job += gridDim.x) {
    const int qi = (int)(job / SLICES);
    const double dp = dpos[qi];
    if (dp < 0) continue;
    const long long W = (long long)SLICES * (blockDim.x / 64);
    const long long w = (job % SLICES) * (long long)(blockDim.x / 64) + (threadIdx.x >> 6);
    const long long p = pos[qi];
    int c = 0;
    for (long long r = w; r < n; r += W) {
      const double d = exact_key(q + (long long)qi * D, g + r * D, D, lane, metric);
      c += (d < dp || (d == dp && g_base + r < p)) ? 1 : 0;
    }
    if (lane == 0 && c) atomicAdd(cnt + qi, c);
  }
}

// exhaustive exact top-k of the flagged queries (a chunk list could have hidden
// a true top-k item, or the gallery is too small for the lists): every wave
// keeps a sorted (key, index) list of the k best rows it sees, lane i holding
// entry i (k <= 64), inserted by ballot + shuffle; lists to part[q][W][k]
constexpr int KNN_XB = 8;  // workgroups (x 4 waves) per flagged query

__global__ void __launch_bounds__(256) knn_exact_topk_part_kernel(const float* __restrict__ q,
                                                                  const float* __restrict__ g, int D, long long n,
                                                                  int k, int metric, const int* __restrict__ flag,
                                                                  double* __restrict__ pkey,
                                                                  long long* __restrict__ pidx) {
  const int qi = blockIdx.y;
  if (!flag[qi]) return;
  const int lane = threadIdx.x & 63;
  const int W = gridDim.x * 4;
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  double lk = INFINITY;
  long long li = 0x7fffffffffffffffLL;
  for (long long r = w; r < n; r += W) {
    const double key = exact_key(q + (long long)qi * D, g + r * D, D, lane, metric);
    const double kk = __shfl(lk, k - 1, 64);
    const long long ki = __shfl(li, k - 1, 64);
    if (key < kk || (key == kk && r < ki)) {  // wave-uniform
      const bool before = lane < k && (lk < key || (lk == key && li < r));
      const int at = __popcll(__builtin_amdgcn_ballot_w64(before));
      const double uk = __shfl_up(lk, 1, 64);
      const long long ui = __shfl_up(li, 1, 64);
      if (lane == at) {
        lk = key;
        li = r;
      } else if (lane > at && lane < k) {
        lk = uk;
        li = ui;
      }
    }
  }
  if (lane < k) {
    const long long o = ((long long)qi * W + w) * k + lane;
    pkey[o] = lk;
    pidx[o] = li == 0x7fffffffffffffffLL ? -1 : li;
  }
}

// k smallest (key, index) of nl lists of k entries (index -1 = empty) -> out;
// one workgroup per row of lists; rows with flag == 0 are left alone (flag ==
// nullptr: every row).  Shared by the flagged-query fallback and
// artsbir_topk_merge (per-shard top-k lists of a sharded gallery).
// Entry j of list l of row qi is at qi * s_row + l * s_list + j.
__global__ void __launch_bounds__(256) topk_lists_merge_kernel(const double* __restrict__ key,
                                                               const long long* __restrict__ idx, int nl, int k,
                                                               long long s_row, long long s_list,
                                                               const int* __restrict__ flag, long long idx_base,
                                                               long long* __restrict__ out_i,
                                                               double* __restrict__ out_d) {
  const int qi = blockIdx.x;
  if (flag && !flag[qi]) return;
  extern __shared__ char sm[];
  unsigned char* used = reinterpret_cast<unsigned char*>(sm);
  const int nc = nl * k;
  const double* kr = key + (long long)qi * s_row;
  const long long* ir = idx + (long long)qi * s_row;
  auto at = [&](int c) { return (long long)(c / k) * s_list + (c % k); };
  for (int c = threadIdx.x; c < nc; c += blockDim.x) used[c] = ir[at(c)] < 0 ? 1 : 0;
  __syncthreads();
  __shared__ double rd[4];
  __shared__ long long ri[4];
  __shared__ int rs[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int r = 0; r < k; ++r) {
    double bd = INFINITY;
    long long bi = 0x7fffffffffffffffLL;
    int bs = -1;
    for (int c = threadIdx.x; c < nc; c += blockDim.x) {
      if (used[c]) continue;
      const double d = kr[at(c)];
      const long long i = ir[at(c)];
      if (bs < 0 || d < bd || (d == bd && i < bi)) { bd = d; bi = i; bs = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double od = __shfl_xor(bd, o, 64);
      const long long oi = __shfl_xor(bi, o, 64);
      const int os = __shfl_xor(bs, o, 64);
      if (os >= 0 && (bs < 0 || od < bd || (od == bd && oi < bi))) { bd = od; bi = oi; bs = os; }
    }
    if (lane == 0) { rd[wid] = bd; ri[wid] = bi; rs[wid] = bs; }
    __syncthreads();
    if (threadIdx.x == 0) {
      double b = rd[0];
      long long bi2 = ri[0];
      int bs2 = rs[0];
      for (int w = 1; w < (int)blockDim.x / 64; ++w)
        if (rs[w] >= 0 && (bs2 < 0 || rd[w] < b || (rd[w] == b && ri[w] < bi2))) { b = rd[w]; bi2 = ri[w]; bs2 = rs[w]; }
      out_i[(long long)qi * k + r] = bs2 >= 0 ? idx_base + bi2 : -1;
      out_d[(long long)qi * k + r] = bs2 >= 0 ? b : INFINITY;
      if (bs2 >= 0) used[bs2] = 1;
    }
    __syncthreads();
  }
}

// exact key of every query's positive when it lies in this shard's rows
// [g_base, g_base + n), else -1 (one wave per query)
__global__ void positive_key_kernel(const float* __restrict__ q, const float* __restrict__ g, int D, int nq,
                                    const long long* __restrict__ pos, long long g_base, long long n, int metric,
                                    double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int qi = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (qi >= nq) return;
  const long long p = pos[qi];
  if (p < g_base || p >= g_base + n) {
    if (lane == 0) out[qi] = -1.0;
    return;
  }
  const double d = exact_key(q + (long long)qi * D, g + (p - g_base) * D, D, lane, metric);
  if (lane == 0) out[qi] = d;
}

__global__ void rank_out_kernel(const int* __restrict__ cnt, int nq, long long* __restrict__ out) {
  const int qi = blockIdx.x * blockDim.x + threadIdx.x;
  if (qi < nq) out[qi] = cnt[qi];
}

}  // namespace artsbir

using namespace artsbir;

extern "C" int artsbir_pairwise_l2(const float* x1, long long n1, const float* x2, long long n2, int D, float eps,
                                   float* out, void* stream) {
  if (!(n1 == n2 || n1 == 1 || n2 == 1)) { set_error("pairwise_l2: shapes %lld vs %lld", n1, n2); return -1; }
  const long long n = n1 > n2 ? n1 : n2;
  long long grid = (n + 3) / 4;
  if (grid > 65536) grid = 65536;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(pairwise_l2_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, x1, n1, x2, n2, D, eps, out);
  ARTSBIR_CHECK_LAUNCH("pairwise_l2");
  return 0;
}

extern "C" int artsbir_rows_prep(int dtype, const float* x, int n, int D, float* sq, void* xc, int ldc, void* stream) {
  const unsigned grid = (unsigned)((n + 3) / 4);
  if (n <= 0) return 0;
  if (ldc < D) ldc = D;
  if (dtype == ARTSBIR_DT_BF16)
    hipLaunchKernelGGL(rows_prep_kernel<bf16>, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, n, D, sq, (bf16*)xc, ldc, 0);
  else
    hipLaunchKernelGGL(rows_prep_kernel<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, n, D, sq, (float*)xc, ldc, 0);
  ARTSBIR_CHECK_LAUNCH("rows_prep");
  return 0;
}

extern "C" int artsbir_knn_band(const float* q, const float* g, const long long* pos, long long g_base, long long n_g,
                                const float* qsq, float gsq_max, int nq, int D, float rel, double* dpos, float* lo,
                                float* hi, void* stream) {
  if (nq <= 0) return 0;
  hipLaunchKernelGGL(knn_band_kernel, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, (hipStream_t)stream, q, g, pos, g_base,
                     n_g, qsq, gsq_max, nq, D, rel, dpos, lo, hi, 0, nullptr);
  ARTSBIR_CHECK_LAUNCH("knn_band");
  return 0;
}

extern "C" int artsbir_knn_band_from_dpos(const double* dpos, const float* qsq, float gsq_max, int nq, float rel,
                                          float* lo, float* hi, void* stream) {
  if (nq <= 0) return 0;
  hipLaunchKernelGGL(knn_band_from_dpos_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     dpos, qsq, gsq_max, nq, rel, lo, hi);
  ARTSBIR_CHECK_LAUNCH("knn_band_from_dpos");
  return 0;
}

extern "C" int artsbir_knn_candidates_per_query(int ng, int tiles_per_chunk) {
  const int tiles = (ng + 127) / 128;
  const int nchunks = (tiles + tiles_per_chunk - 1) / tiles_per_chunk;
  return nchunks * KT;
}

extern "C" int artsbir_knn_scan(int dtype, const void* qc, const void* gc, const float* qsq, const float* gsq, int nq,
                                int ng, int D, int tiles_per_chunk, const float* lo, const float* hi, int* cnt, int* unc,
                                int unc_cap, float* cand_d, int* cand_i, void* stream) {
  const int EPC = dtype == ARTSBIR_DT_BF16 ? 8 : 4;
  if (D % (8 * EPC)) { set_error("knn_scan: D=%d must be a multiple of %d", D, 8 * EPC); return -1; }
  if (nq <= 0 || ng <= 0) return 0;
  KnnScanArgs a;
  a.q = qc; a.g = gc; a.qsq = qsq; a.gsq = gsq; a.gsq_max = 0.f; a.gsq_max_p = nullptr; a.thr0 = nullptr; a.kb = nullptr; a.hist = nullptr; a.hbase = nullptr; a.kq = 0; a.rel = 0.f; a.Nq = nq; a.Ng = ng; a.D = D;
  a.tiles_per_chunk = tiles_per_chunk;
  const int tiles = (ng + 127) / 128;
  a.nchunks = (tiles + tiles_per_chunk - 1) / tiles_per_chunk;
  a.lo = lo; a.hi = hi; a.cnt = cnt; a.unc = unc; a.unc_cap = unc_cap; a.cand_d = cand_d; a.cand_i = cand_i;
  const unsigned grid = (unsigned)(a.nchunks * ((nq + 127) / 128));
  if (dtype == ARTSBIR_DT_BF16)
    hipLaunchKernelGGL(knn_scan_kernel<bf16>, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(knn_scan_kernel<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
  ARTSBIR_CHECK_LAUNCH("knn_scan");
  return 0;
}

extern "C" int artsbir_knn_merge(const float* q, const float* g, int D, int nq, int nchunks, const float* cand_d,
                                 const int* cand_i, const float* qsq, float gsq_max, float rel, long long g_base, int k,
                                 long long* out_i, double* out_d, int* flag, void* stream) {
  if (nq <= 0) return 0;
  if (k > nchunks * KT) { set_error("knn_merge: k=%d exceeds candidates %d", k, nchunks * KT); return -1; }
  const size_t sh = (size_t)nchunks * KT * (sizeof(double) + sizeof(int));
  if (sh > 60000) { set_error("knn_merge: too many candidates (%d chunks)", nchunks); return -1; }
  if (!launch_merge_wave(nq, (hipStream_t)stream, q, g, D, nchunks, cand_d, cand_i, qsq, gsq_max, rel, g_base, k, out_i,
                         out_d, flag, 0, nullptr, 0LL))
    hipLaunchKernelGGL(knn_merge_kernel, dim3(nq), dim3(256), sh, (hipStream_t)stream, q, g, D, nchunks, cand_d, cand_i,
                       qsq, gsq_max, rel, g_base, k, out_i, out_d, flag, 0, nullptr, 0LL);
  ARTSBIR_CHECK_LAUNCH("knn_merge");
  return 0;
}

extern "C" int artsbir_knn_uncertain(const float* q, const float* g, int D, const int* unc, int unc_cap,
                                     const double* dpos, const long long* pos, long long g_base, int* cnt, void* stream) {
  hipLaunchKernelGGL(knn_uncertain_kernel, dim3(1024), dim3(256), 0, (hipStream_t)stream, q, g, D, unc, unc_cap, dpos,
                     pos, g_base, cnt, 0);
  ARTSBIR_CHECK_LAUNCH("knn_uncertain");
  return 0;
}

extern "C" int artsbir_knn_exact_all(const float* q, const float* g, int D, int n, double* out, void* stream) {
  if (n <= 0) return 0;
  unsigned grid = (unsigned)((n + 3) / 4);
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(knn_exact_all_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, q, g, D, n, out, 0);
  ARTSBIR_CHECK_LAUNCH("knn_exact_all");
  return 0;
}

extern "C" int artsbir_rows_prep_aug(const float* x, int n, int D, int Dp, float* sq, void* xa, void* stream) {
  if (Dp < D || Dp % 16) { set_error("rows_prep_aug: Dp=%d must be >= D=%d and a multiple of 16", Dp, D); return -1; }
  if (n <= 0) return 0;
  hipLaunchKernelGGL(rows_prep_aug_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x, n, D, Dp,
                     sq, (bf16*)xa, 0);
  ARTSBIR_CHECK_LAUNCH("rows_prep_aug");
  return 0;
}

extern "C" int artsbir_knn_scan_aug_supported(int Dp) { return Dp == 64 || Dp == 128 || Dp == 256 || Dp == 512; }

extern "C" int artsbir_knn_scan_aug(const void* qc, const void* ga, const float* qsq, float gsq_max, int nq, int ng,
                                    int Dp, int tiles_per_chunk, const float* thr0, unsigned* kbound, int k, float rel,
                                    const float* lo, const float* hi, int* cnt, int* unc, int unc_cap, float* cand_d,
                                    int* cand_i, void* stream) {
  if (!artsbir_knn_scan_aug_supported(Dp)) { set_error("knn_scan_aug: Dp=%d not in {64,128,256,512}", Dp); return -1; }
  if (tiles_per_chunk <= 0 || (long long)tiles_per_chunk * 128 * (2LL * Dp + 16) > 0x7fffffffLL) {
    set_error("knn_scan_aug: tiles_per_chunk=%d out of range", tiles_per_chunk);
    return -1;
  }
  if (kbound && (k < 1 || k > KT)) { set_error("knn_scan_aug: k=%d must be in 1..%d with a shared bound", k, KT); return -1; }
  if (nq <= 0 || ng <= 0) return 0;
  KnnScanArgs a;
  a.q = qc; a.g = ga; a.qsq = qsq; a.gsq = nullptr; a.gsq_max = gsq_max; a.gsq_max_p = nullptr; a.thr0 = thr0; a.kb = kbound; a.hist = nullptr; a.hbase = nullptr; a.kq = k; a.rel = rel; a.Nq = nq; a.Ng = ng; a.D = Dp;
  a.tiles_per_chunk = tiles_per_chunk;
  const int tiles = (ng + 127) / 128;
  a.nchunks = (tiles + tiles_per_chunk - 1) / tiles_per_chunk;
  a.lo = lo; a.hi = hi; a.cnt = cnt; a.unc = unc; a.unc_cap = unc_cap; a.cand_d = cand_d; a.cand_i = cand_i;
  const unsigned grid = (unsigned)(a.nchunks * ((nq + 255) / 256));
  knn_scan_v2_launch(Dp, grid, a, 0, (hipStream_t)stream);
  ARTSBIR_CHECK_LAUNCH("knn_scan_aug");
  return 0;
}

// ---------------------------------------------------------------------------
// One-call exact top-k + rank of the positive (the drop-in for the per-query
// loop of inference.py:30-69: utils.euclidean_distance / cosine_distance of
// [1,D] vs [N,D], topk(N) -> position of the positive, topk(k)).  Launch
// sequence (all on `stream`, no host synchronisation):
//   rows_prep(q), rows_prep_aug(g) [unit rows for cosine] -> min/max |g|^2 ->
//   per-query eps + dpos init -> band (exact key of the positive) -> MFMA scan
//   -> exact merge -> uncertain checks -> overflow recount -> exhaustive top-k
//   of flagged queries -> ranks.
namespace {
// optional HIP-event timing of the scan kernel inside artsbir_pairwise_l2_topk
// (bench.py prices the scan against the MFMA roof with it)
int g_scan_prof = 0;
std::vector<std::pair<hipEvent_t, hipEvent_t>> g_scan_ev;

struct TopkPlan {
  int dtype, v2, Dp, tpc, nchunks, ncand, unc_cap;
  int ncand_alloc;  // candidate slots the workspace holds per query (>= ncand)
  size_t off[20];
  size_t total;
};
constexpr int TOPK_KMAX = 64;
int g_topk_unc_cap = 1 << 20;  // artsbir_knn_set_unc_cap (tests force the overflow path)

enum { W_QSQ, W_GSQ, W_EXT, W_QEPS, W_QC, W_GC, W_LO, W_HI, W_DPOS, W_CNT, W_UNC, W_CD, W_CI, W_FLAG, W_PK, W_PI, W_KB,
       W_HB, W_HIST, W_END };

int topk_plan(int dtype, int Q, long long N, int D, int k, int tpc_req, TopkPlan& p) {
  if (Q < 0 || N < 1 || D < 1 || k < 1 || k > TOPK_KMAX || N > 0x7fffffffLL) {
    set_error("pairwise_l2_topk: need Q >= 0, 1 <= N < 2^31, D >= 1, 1 <= k <= %d (Q=%d N=%lld D=%d k=%d)", TOPK_KMAX,
              Q, N, D, k);
    return -1;
  }
  if (dtype != ARTSBIR_DT_BF16 && dtype != ARTSBIR_DT_F32) { set_error("pairwise_l2_topk: dtype %d", dtype); return -1; }
  p.dtype = dtype;
  const int step = dtype == ARTSBIR_DT_BF16 ? 64 : 32;
  p.Dp = (D + step - 1) / step * step;
  p.v2 = dtype == ARTSBIR_DT_BF16 && artsbir_knn_scan_aug_supported(p.Dp);
  const long long tiles = (N + 127) / 128;
  long long tpc = tpc_req > 0 ? tpc_req : (p.v2 ? 256 : 64);
  const long long need = (k + KT - 1) / KT;           // chunks whose lists can hold k items
  if (tiles / need < tpc) tpc = tiles / need > 0 ? tiles / need : 1;
  const long long maxch = 60000 / (KT * 12);          // knn_merge's shared memory
  if ((tiles + tpc - 1) / tpc > maxch) tpc = (tiles + maxch - 1) / maxch;
  static const bool balance = [] { const char* e = getenv("ARTSBIR_KNN_BALANCE"); return !e || atoi(e) != 0; }();
  // the workspace is laid out for the most chunks the balancing below may pick,
  // whatever the device it finds (or none, as in a host-side workspace query):
  // the layout depends on the arguments alone
  long long nch_alloc = (tiles + tpc - 1) / tpc;
  if (tpc_req <= 0 && p.v2) {
    const long long tmin = (tpc * 3 + 3) / 4 > 0 ? (tpc * 3 + 3) / 4 : 1;
    const long long nmax = (tiles + tmin - 1) / tmin;
    nch_alloc = std::max(nch_alloc, std::min(nmax, maxch));
  }
  if (tpc_req <= 0 && p.v2 && Q > 0 && balance) {
    // the v2 scan runs ceil(Q / 256) query tiles x nchunks workgroups, one per CU
    // (140 KB of LDS): take the chunk length (at most 1/4 shorter) whose grid
    // fills its last round of workgroups.  C4 (10k x 1M): 31 chunks of 256
    // tiles = 1240 workgroups, 4.84 rounds on 256 CUs, the last chunk half
    // full; 32 chunks of 245 tiles = 1280 = 5.00 rounds of 245 tiles
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu > 0) {
      const long long ntq = (Q + 255) / 256;
      long long best = tpc, bestc = -1;
      for (long long t = tpc; t >= (tpc * 3 + 3) / 4 && t >= 1; --t) {
        const long long nch = (tiles + t - 1) / t;
        if (nch > maxch || tiles / need < t) continue;
        const long long cost = (ntq * nch + ncu - 1) / ncu * t;  // rounds x tiles per workgroup
        if (bestc < 0 || cost < bestc) { bestc = cost; best = t; }
      }
      tpc = best;
    }
  }
  p.tpc = (int)tpc;
  p.nchunks = (int)((tiles + tpc - 1) / tpc);
  p.ncand = p.nchunks * KT;
  p.ncand_alloc = (int)std::max<long long>(p.nchunks, nch_alloc) * KT;
  p.unc_cap = g_topk_unc_cap;
  const size_t es = dtype == ARTSBIR_DT_BF16 ? 2 : 4;
  const size_t W = KNN_XB * 4;
  size_t sz[W_END];
  sz[W_QSQ] = 4 * (size_t)Q;
  sz[W_GSQ] = 4 * (size_t)N;
  sz[W_EXT] = 8;
  sz[W_QEPS] = 4 * (size_t)Q;
  sz[W_QC] = (size_t)Q * p.Dp * es;
  sz[W_GC] = p.v2 ? (size_t)N * (p.Dp + 8) * 2 : (size_t)N * p.Dp * es;
  sz[W_LO] = sz[W_HI] = 4 * (size_t)Q;
  sz[W_DPOS] = 8 * (size_t)Q;
  sz[W_CNT] = 4 * (size_t)Q;
  sz[W_UNC] = 4 * (2 * (size_t)p.unc_cap + 1);
  sz[W_CD] = sz[W_CI] = 4 * (size_t)Q * p.ncand_alloc;
  sz[W_FLAG] = 4 * (size_t)Q;
  sz[W_PK] = sz[W_PI] = 8 * (size_t)Q * W * k;
  sz[W_KB] = 4 * (size_t)Q;
  sz[W_HB] = 4 * (size_t)Q;
  sz[W_HIST] = 4 * (size_t)Q * HB_BINS;
  size_t o = 0;
  for (int i = 0; i < W_END; ++i) {
    p.off[i] = o;
    o += (sz[i] + 255) / 256 * 256;
  }
  p.total = o;
  return 0;
}
}  // namespace

extern "C" int artsbir_knn_stat_read(unsigned long long* out4, int reset) {
  if (hipMemcpyFromSymbol(out4, HIP_SYMBOL(g_knn_stat), sizeof(unsigned long long) * 4) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long z[4] = {0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_knn_stat), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}

extern "C" long long artsbir_pairwise_l2_topk_workspace(int dtype, int Q, long long N, int D, int k,
                                                        int tiles_per_chunk) {
  TopkPlan p;
  if (topk_plan(dtype, Q, N, D, k, tiles_per_chunk, p)) return -1;
  return (long long)p.total;
}

extern "C" int artsbir_pairwise_l2_topk(int dtype, int metric, const float* q, int Q, const float* g, long long N, int D,
                                        int k, const long long* positives, const double* dpos_in, long long g_base,
                                        int tiles_per_chunk, long long* out_idx, double* out_dist, long long* out_rank,
                                        double* out_dpos, void* workspace, long long workspace_bytes, void* stream) {
  if (metric != 0 && metric != 1) { set_error("pairwise_l2_topk: metric %d (0 = euclidean, 1 = cosine)", metric); return -1; }
  TopkPlan p;
  if (topk_plan(dtype, Q, N, D, k, tiles_per_chunk, p)) return -1;
  if (!workspace || workspace_bytes < (long long)p.total) {
    set_error("pairwise_l2_topk: workspace of %lld bytes < %zu needed", workspace_bytes, p.total);
    return -1;
  }
  if (!q || !g || !out_idx || !out_dist) { set_error("pairwise_l2_topk: null input/output"); return -1; }
  if (out_rank && !positives) { set_error("pairwise_l2_topk: ranks need positives"); return -1; }
  if (Q == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  char* w = static_cast<char*>(workspace);
  float* qsq = reinterpret_cast<float*>(w + p.off[W_QSQ]);
  float* gsq = reinterpret_cast<float*>(w + p.off[W_GSQ]);
  unsigned* ext = reinterpret_cast<unsigned*>(w + p.off[W_EXT]);
  float* qeps = reinterpret_cast<float*>(w + p.off[W_QEPS]);
  void* qc = w + p.off[W_QC];
  void* gc = w + p.off[W_GC];
  float* lo = reinterpret_cast<float*>(w + p.off[W_LO]);
  float* hi = reinterpret_cast<float*>(w + p.off[W_HI]);
  double* dpos = reinterpret_cast<double*>(w + p.off[W_DPOS]);
  int* cnt = reinterpret_cast<int*>(w + p.off[W_CNT]);
  int* unc = reinterpret_cast<int*>(w + p.off[W_UNC]);
  float* cand_d = reinterpret_cast<float*>(w + p.off[W_CD]);
  int* cand_i = reinterpret_cast<int*>(w + p.off[W_CI]);
  int* flag = reinterpret_cast<int*>(w + p.off[W_FLAG]);
  double* pkey = reinterpret_cast<double*>(w + p.off[W_PK]);
  long long* pidx = reinterpret_cast<long long*>(w + p.off[W_PI]);
  unsigned* kbuf = reinterpret_cast<unsigned*>(w + p.off[W_KB]);
  static const bool kb_on = [] { const char* e = getenv("ARTSBIR_KNN_KB"); return !e || atoi(e) != 0; }();
  // the published-item histogram tightening kb (ARTSBIR_KNN_HIST=0: kb from each chunk's own k-th only)
  static const bool hist_on = [] { const char* e = getenv("ARTSBIR_KNN_HIST"); return !e || atoi(e) != 0; }();
  unsigned* hbase = reinterpret_cast<unsigned*>(w + p.off[W_HB]);
  unsigned* hist = reinterpret_cast<unsigned*>(w + p.off[W_HIST]);
  const int ng = (int)N;
  const float rel = dtype == ARTSBIR_DT_BF16 ? (float)(0x1p-6 + 0x1p-12) : (float)0x1p-14;

  if (hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(ext), 0, 1, st) != hipSuccess ||
      hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(ext + 1), 0x7f800000, 1, st) != hipSuccess ||
      hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(kbuf), (int)0xff800000u, Q, st) != hipSuccess ||  // kb_enc(+inf)
      hipMemsetAsync(w + p.off[W_HB], 0, p.off[W_HIST] - p.off[W_HB] + 4 * (size_t)Q * HB_BINS, st) != hipSuccess) {
    set_error("pairwise_l2_topk: memset failed");
    return -2;
  }
  const unsigned gq = (unsigned)((Q + 3) / 4), gg = (unsigned)((N + 3) / 4);
  if (dtype == ARTSBIR_DT_BF16)
    hipLaunchKernelGGL(rows_prep_kernel<bf16>, dim3(gq), dim3(256), 0, st, q, Q, D, qsq, (bf16*)qc, p.Dp, metric);
  else
    hipLaunchKernelGGL(rows_prep_kernel<float>, dim3(gq), dim3(256), 0, st, q, Q, D, qsq, (float*)qc, p.Dp, metric);
  if (p.v2)
    hipLaunchKernelGGL(rows_prep_aug_kernel, dim3(gg), dim3(256), 0, st, g, ng, D, p.Dp, gsq, (bf16*)gc, metric);
  else if (dtype == ARTSBIR_DT_BF16)
    hipLaunchKernelGGL(rows_prep_kernel<bf16>, dim3(gg), dim3(256), 0, st, g, ng, D, gsq, (bf16*)gc, p.Dp, metric);
  else
    hipLaunchKernelGGL(rows_prep_kernel<float>, dim3(gg), dim3(256), 0, st, g, ng, D, gsq, (float*)gc, p.Dp, metric);
  {
    long long b = (N + 255) / 256;
    if (b > 256) b = 256;
    hipLaunchKernelGGL(sq_minmax_kernel, dim3((unsigned)b), dim3(256), 0, st, gsq, N, ext);
  }
  hipLaunchKernelGGL(knn_init_kernel, dim3((unsigned)((Q + 255) / 256)), dim3(256), 0, st, qsq, ext, Q, rel, metric,
                     dpos_in, qeps, dpos, cnt, unc + 2 * p.unc_cap);
  if (positives)
    hipLaunchKernelGGL(knn_band_kernel, dim3(gq), dim3(256), 0, st, q, g, positives, g_base, N, qsq, 0.f, Q, D, rel, dpos,
                       lo, hi, metric, qeps);
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  if (g_scan_prof && hipEventCreate(&ev0) == hipSuccess && hipEventCreate(&ev1) == hipSuccess) {
    (void)hipEventRecord(ev0, st);
    g_scan_ev.emplace_back(ev0, ev1);
  }
  KnnScanArgs a;
  a.q = qc; a.g = gc; a.qsq = qsq; a.gsq = gsq; a.gsq_max = 0.f; a.gsq_max_p = reinterpret_cast<const float*>(ext);
  a.thr0 = nullptr; a.kb = (p.v2 && kb_on) ? kbuf : nullptr; a.kq = k;
  a.hist = a.kb && hist_on ? hist : nullptr; a.hbase = a.hist ? hbase : nullptr; a.rel = rel; a.Nq = Q; a.Ng = ng; a.D = p.Dp;
  a.tiles_per_chunk = p.tpc;
  a.nchunks = p.nchunks;
  a.lo = positives ? lo : nullptr; a.hi = positives ? hi : nullptr;
  a.cnt = cnt; a.unc = unc; a.unc_cap = p.unc_cap; a.cand_d = cand_d; a.cand_i = cand_i;
  if (p.v2) {
    const unsigned grid = (unsigned)(p.nchunks * ((Q + 255) / 256));
    const int sstat = knn_stat_on() ? 1 : 0;
    knn_scan_v2_launch(p.Dp, grid, a, sstat, st);
    set_last_kernel("knn_scan_v2_kernel");
  } else {
    // knn_scan_kernel's chunks are tiles_per_chunk x 128 rows as well
    const unsigned grid = (unsigned)(p.nchunks * ((Q + 127) / 128));
    if (dtype == ARTSBIR_DT_BF16)
      hipLaunchKernelGGL(knn_scan_kernel<bf16>, dim3(grid), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL(knn_scan_kernel<float>, dim3(grid), dim3(256), 0, st, a);
    set_last_kernel("knn_scan_kernel");
  }
  ARTSBIR_CHECK_LAUNCH("pairwise_l2_topk scan");
  if (ev1) (void)hipEventRecord(ev1, st);
  const size_t sh = (size_t)p.ncand * (sizeof(double) + sizeof(int));
  if (!launch_merge_wave(Q, st, q, g, D, p.nchunks, cand_d, cand_i, qsq, 0.f, rel, g_base, k, out_idx, out_dist, flag,
                         metric, qeps, N))
    hipLaunchKernelGGL(knn_merge_kernel, dim3(Q), dim3(256), sh, st, q, g, D, p.nchunks, cand_d, cand_i, qsq, 0.f, rel,
                       g_base, k, out_idx, out_dist, flag, metric, qeps, N);
  if (positives) {
    hipLaunchKernelGGL(knn_uncertain_kernel, dim3(1024), dim3(256), 0, st, q, g, D, unc, p.unc_cap, dpos, positives,
                       g_base, cnt, metric);
    hipLaunchKernelGGL(knn_count_reset_kernel, dim3((unsigned)((Q + 255) / 256)), dim3(256), 0, st,
                       unc + 2 * p.unc_cap, p.unc_cap, Q, cnt);
    hipLaunchKernelGGL(knn_count_exhaustive_kernel, dim3(2048), dim3(256), 0, st, q, g, D, N, unc + 2 * p.unc_cap,
                       p.unc_cap, dpos, positives, g_base, cnt, metric, Q);
  }
  hipLaunchKernelGGL(knn_exact_topk_part_kernel, dim3(KNN_XB, Q), dim3(256), 0, st, q, g, D, N, k, metric, flag, pkey,
                     pidx);
  hipLaunchKernelGGL(topk_lists_merge_kernel, dim3(Q), dim3(256), (size_t)KNN_XB * 4 * k, st, pkey, pidx,
                     KNN_XB * 4, k, (long long)KNN_XB * 4 * k, (long long)k, flag, g_base, out_idx, out_dist);
  if (out_rank) hipLaunchKernelGGL(rank_out_kernel, dim3((unsigned)((Q + 255) / 256)), dim3(256), 0, st, cnt, Q, out_rank);
  if (out_dpos && hipMemcpyAsync(out_dpos, dpos, 8 * (size_t)Q, hipMemcpyDeviceToDevice, st) != hipSuccess) {
    set_error("pairwise_l2_topk: dpos copy failed");
    return -2;
  }
  ARTSBIR_CHECK_LAUNCH("pairwise_l2_topk");
  return 0;
}

// per-shard top-k lists [nshard][Q][k] (as gathered from the ranks, index -1 =
// empty) -> the global top-k by (distance, index); replaces the host-side sort
// of the gathered lists (inference.py:49,65 topk on the whole gallery)
extern "C" int artsbir_topk_merge(int nshard, int Q, int k, const double* dist, const long long* idx,
                                  long long* out_idx, double* out_dist, void* stream) {
  if (nshard < 1 || k < 1 || Q < 0 || (long long)nshard * k > 65536) {
    set_error("topk_merge: nshard=%d k=%d Q=%d", nshard, k, Q);
    return -1;
  }
  if (Q == 0) return 0;
  hipLaunchKernelGGL(topk_lists_merge_kernel, dim3(Q), dim3(256), (size_t)nshard * k, (hipStream_t)stream, dist, idx,
                     nshard, k, (long long)k, (long long)Q * k, (const int*)nullptr, 0LL, out_idx, out_dist);
  ARTSBIR_CHECK_LAUNCH("topk_merge");
  return 0;
}

extern "C" int artsbir_positive_key(int metric, const float* q, int Q, const float* g, long long n, int D,
                                    const long long* pos, long long g_base, double* out, void* stream) {
  if (metric != 0 && metric != 1) { set_error("positive_key: metric %d", metric); return -1; }
  if (Q <= 0) return 0;
  hipLaunchKernelGGL(positive_key_kernel, dim3((unsigned)((Q + 3) / 4)), dim3(256), 0, (hipStream_t)stream, q, g, D, Q,
                     pos, g_base, n, metric, out);
  ARTSBIR_CHECK_LAUNCH("positive_key");
  return 0;
}

// scan-kernel timing of artsbir_pairwise_l2_topk: on = 1 starts collecting (and
// drops what was collected), 0 stops; read waits for the recorded events and
// returns the summed scan time (ms) and the number of scans.
extern "C" int artsbir_scan_profile(int on) {
  for (auto& e : g_scan_ev) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  g_scan_ev.clear();
  g_scan_prof = on;
  return 0;
}

extern "C" int artsbir_scan_profile_read(double* total_ms, int* count) {
  double t = 0.0;
  int n = 0;
  for (auto& e : g_scan_ev) {
    if (hipEventSynchronize(e.second) != hipSuccess) { set_error("scan_profile_read: event sync failed"); return -2; }
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e.first, e.second) == hipSuccess) { t += ms; ++n; }
  }
  *total_ms = t;
  *count = n;
  return 0;
}

// capacity of the uncertain-item queue of artsbir_pairwise_l2_topk (default
// 2^20); a small value forces the exhaustive recount path (tests).  Returns the old one.
extern "C" int artsbir_knn_set_unc_cap(int cap) {
  const int old = g_topk_unc_cap;
  if (cap > 0) g_topk_unc_cap = cap;
  return old;
}
