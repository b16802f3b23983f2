// Smoothed-aggregation algebraic multigrid for the unstructured (general
// hexahedral / quadrilateral) meshes: the grid-operator kernels of the
// V-cycle (gfx950).  The hierarchy is built once on the host (tv_amg.cpp)
// from the T-independent cell operator; it replaces the reference's PCGAMG
// (ThermoViscoProblem.py:343-346) on the meshes the box multigrid cannot
// coarsen.
//
// Every operator -- coarse A_l, prolongation P_l, restriction R_l = P_l^T --
// is a SELL-64 matrix (one 64-row slice per wavefront, column-major inside
// the slice, as the fine operator of tv_um.hip), and every kernel is one
// lane per row with a contiguous slice range per wave.  Bytes per stored
// entry: 12 (value + column) + the gathered vector entry (cached).
#include <algorithm>

#include "tv_device.h"

namespace tv {
namespace {

enum AmgMode {
  AMG_APPLY = 0,     // y = A x
  AMG_RESTRICT = 1,  // y = R (x - x2)  [x2 optional]; y2 = omega dinv y (next level's pre-smoothing from 0)
  AMG_PROLONG = 2,   // y = x2 + P x (x2 may alias y: each row reads its own entry only)
  AMG_POST = 3,      // y = x2 + omega dinv (b - A x2)  (x = x2: the smoothed iterate's own operator product)
  AMG_PROLONG0 = 4,  // level 0, additive: z = x2 + P x, (z.z, z.b) records + the KSPCG tail
};

constexpr int kAmgBlocksMax = 2048;

// the sum over row r of M of val * (x - x2)[col] (x2 optional): SELL-64 (lane
// = row of the wave's slice, column-major entries) or CSR (one row per lane,
// the transfers' short rows: no slice padding); U entries in flight per lane
template <typename V>
__device__ __forceinline__ double row_sum(const Sell& M, int64_t r, const double* __restrict__ x,
                                          const double* __restrict__ x2) {
  int64_t k0, step;
  int len;
  if (M.csr) {
    k0 = M.soff[r];
    len = (int)(M.soff[r + 1] - k0);
    step = 1;
  } else {
    const int64_t s = r >> 6;
    k0 = M.soff[s] + (r & 63);
    len = (int)((M.soff[s + 1] - M.soff[s]) >> 6);
    step = 64;
  }
  const int* __restrict__ cs = M.cols + k0;
  const V* __restrict__ vs = reinterpret_cast<const V*>(M.vals) + k0;
  constexpr int U = 8;
  double acc = 0.0;
  for (int k = 0; k < len; k += U) {
    int c[U];
    double a[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const bool ok = k + j < len;
      const int64_t o = step * (ok ? k + j : 0);
      c[j] = __builtin_nontemporal_load(&cs[o]);
      a[j] = (double)__builtin_nontemporal_load(&vs[o]);
      if (!ok) a[j] = 0.0;
    }
#pragma unroll
    for (int j = 0; j < U; ++j) acc += a[j] * (x2 ? x[c[j]] - x2[c[j]] : x[c[j]]);
  }
  return acc;
}

template <int MODE, typename V>
__global__ __launch_bounds__(kBlock) void k_amg_rows(Sell M, const PcgState* __restrict__ st,
                                                     const double* __restrict__ x, const double* x2,
                                                     const double* __restrict__ b, const double* __restrict__ dinv,
                                                     double omega, double* y, double* __restrict__ y2,
                                                     double* __restrict__ partials, RedTail rt) {
  if (st != nullptr && st->done) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int WPB = kBlock / 64;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  double zz = 0.0, zb = 0.0;
  // q: the row's position in the stored layout; r: the row (perm: SELL rows
  // sorted by length inside windows, so a slice's rows have similar lengths)
  auto row = [&](int64_t q) {
    const double acc = row_sum<V>(M, q, (MODE == AMG_POST) ? x2 : x, (MODE == AMG_RESTRICT) ? x2 : nullptr);
    const int64_t r = M.perm ? (int64_t)M.perm[q] : q;
    if (MODE == AMG_APPLY) {
      y[r] = acc;
    } else if (MODE == AMG_RESTRICT) {
      y[r] = acc;
      if (y2) y2[r] = omega * dinv[r] * acc;
    } else if (MODE == AMG_PROLONG) {
      y[r] = x2[r] + acc;
    } else if (MODE == AMG_POST) {
      y[r] = x2[r] + omega * dinv[r] * (b[r] - acc);
    } else {
      const double z = x2[r] + acc;
      y[r] = z;
      zz += z * z;
      zb += z * b[r];
    }
  };
  if (M.csr) {  // a contiguous row range per workgroup (XCD-remapped)
    const int64_t per = (M.nrow + gridDim.x - 1) / gridDim.x;
    const int64_t r0 = (int64_t)blk * per, r1 = std::min<int64_t>(r0 + per, M.nrow);
    for (int64_t r = r0 + threadIdx.x; r < r1; r += kBlock) row(r);
  } else {  // a contiguous slice range per wave
    const int64_t nw = (int64_t)gridDim.x * WPB;
    const int64_t gw = (int64_t)blk * WPB + wave;
    const int64_t chunk = (M.nslice + nw - 1) / nw;
    const int64_t s0 = gw * chunk, s1 = std::min<int64_t>(s0 + chunk, M.nslice);
    for (int64_t s = s0; s < s1; ++s) {
      const int64_t r = s * 64 + lane;
      if (r < M.nrow) row(r);
    }
  }
  if (MODE == AMG_PROLONG0) {
    __shared__ double red[2][WPB];
    const double s_zz = wave_sum64(zz), s_zb = wave_sum64(zb);
    if (lane == 0) {
      red[0][wave] = s_zz;
      red[1][wave] = s_zb;
    }
    __syncthreads();
    if (threadIdx.x < 2)
      store_partial(&partials[2 * (int64_t)blockIdx.x + threadIdx.x],
                    (red[threadIdx.x][0] + red[threadIdx.x][1]) + (red[threadIdx.x][2] + red[threadIdx.x][3]));
    fused_reduce_tail<2>(rt, gridDim.x);
  }
}

int amg_blocks(const Sell& M) {
  const int64_t units = M.csr ? (M.nrow + kBlock - 1) / kBlock : (M.nslice + 3) / 4;
  return (int)std::max<int64_t>(1, std::min<int64_t>(units, kAmgBlocksMax));
}

template <int MODE>
int launch(const Sell& M, const PcgState* st, const double* x, const double* x2, const double* b, const double* dinv,
           double omega, double* y, double* y2, double* partials, const RedTail* tail, hipStream_t s) {
  const int nb = amg_blocks(M);
  const RedTail rt = tail ? *tail : RedTail{};
  if (M.fp32)
    hipLaunchKernelGGL((k_amg_rows<MODE, float>), dim3(nb), dim3(kBlock), 0, s, M, st, x, x2, b, dinv, omega, y, y2,
                       partials, rt);
  else
    hipLaunchKernelGGL((k_amg_rows<MODE, double>), dim3(nb), dim3(kBlock), 0, s, M, st, x, x2, b, dinv, omega, y, y2,
                       partials, rt);
  return nb;
}

}  // namespace

int amg_num_blocks(const Sell& M) { return amg_blocks(M); }

void launch_amg_apply(const Sell& A, const PcgState* st, const double* x, double* y, hipStream_t s) {
  launch<AMG_APPLY>(A, st, x, nullptr, nullptr, nullptr, 0.0, y, nullptr, nullptr, nullptr, s);
}
void launch_amg_restrict(const Sell& R, const PcgState* st, const double* x, const double* x2, const double* dinv_c,
                         double omega_c, double* b_c, double* x_c, hipStream_t s) {
  launch<AMG_RESTRICT>(R, st, x, x2, nullptr, dinv_c, omega_c, b_c, x_c, nullptr, nullptr, s);
}
void launch_amg_prolong(const Sell& P, const PcgState* st, const double* x_c, const double* x_old, double* x_new,
                        hipStream_t s) {
  launch<AMG_PROLONG>(P, st, x_c, x_old, nullptr, nullptr, 0.0, x_new, nullptr, nullptr, nullptr, s);
}
void launch_amg_post(const Sell& A, const PcgState* st, const double* x, const double* b, const double* dinv,
                     double omega, double* y, hipStream_t s) {
  launch<AMG_POST>(A, st, nullptr, x, b, dinv, omega, y, nullptr, nullptr, nullptr, s);
}
int launch_amg_prolong0(const Sell& P, const PcgState* st, const double* x_c, const double* x0, const double* r,
                        double* z, double* partials, const RedTail* tail, hipStream_t s) {
  return launch<AMG_PROLONG0>(P, st, x_c, x0, r, nullptr, 0.0, z, nullptr, partials, tail, s);
}

}  // namespace tv
