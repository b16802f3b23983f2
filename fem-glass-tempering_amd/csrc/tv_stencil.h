// Device helpers shared by the rectilinear (box) kernels of tv_cg.hip and
// tv_mg.hip: the Robin facet quadrature of the Q1 boundary terms, the 32-bit
// node decode and the closed-form index maps of the box multigrid transfers.
#pragma once
#include "tv_device.h"

namespace tv {
namespace {

enum { MODE_RES = 0, MODE_JAC = 1 };

// 3-point Gauss-Legendre on [0, 1]
__device__ constexpr double kGX[3] = {0.11270166537925831148, 0.5, 0.88729833462074168852};
__device__ constexpr double kGW[3] = {5.0 / 18.0, 8.0 / 18.0, 5.0 / 18.0};

__device__ __forceinline__ double g_rad_conv(const CgGrid& g, double T) {
  const double T2 = T * T;
  return g.a_rad * (T2 * T2 - g.T_amb4) + g.a_conv * (T - g.T_amb);
}
__device__ __forceinline__ double dg_rad_conv(const CgGrid& g, double T) {
  return g.a_rad * 4.0 * (T * T * T) + g.a_conv;
}

// Robin facet contribution at a boundary node.  The node sits at the centre of
// a 3x3 patch over the two tangential axes of its face; patch[u+1][v+1] holds
// the value at tangential offset (u, v).  The up-to-four facets around the node
// are integrated with 3x3 Gauss points; a degenerate tangential axis collapses
// to a point (weight 1, basis 1) so the same code gives the 1D point evaluation
// of ds at the interval end points.
//   MODE_RES: dt * sum_f int_f g(T_h) phi_I
//   MODE_JAC: dt * sum_f int_f g'(T_h) phi_I p_h       (diag: p_h -> phi_I)
template <int MODE, bool DIAG, bool D1, bool D2>
__device__ double facet_sum(const CgGrid& g, double h1lo, double h1hi, double h2lo, double h2hi,
                            const double (&Tp)[3][3], const double (&Pp)[3][3]) {
  double acc = 0.0;
  constexpr int NS1 = D1 ? 1 : 2, NQ1 = D1 ? 1 : 3;
  constexpr int NS2 = D2 ? 1 : 2, NQ2 = D2 ? 1 : 3;
#pragma unroll
  for (int s1 = 0; s1 < NS1; ++s1) {
    const double h1 = D1 ? 1.0 : (s1 == 0 ? h1lo : h1hi);
    if (!D1 && !(h1 > 0.0)) continue;
    const int o1 = D1 ? 0 : (s1 == 0 ? -1 : 1);
#pragma unroll
    for (int s2 = 0; s2 < NS2; ++s2) {
      const double h2 = D2 ? 1.0 : (s2 == 0 ? h2lo : h2hi);
      if (!D2 && !(h2 > 0.0)) continue;
      const int o2 = D2 ? 0 : (s2 == 0 ? -1 : 1);
      const double T00 = Tp[1][1], T10 = Tp[1 + o1][1], T01 = Tp[1][1 + o2], T11 = Tp[1 + o1][1 + o2];
      const double P00 = Pp[1][1], P10 = Pp[1 + o1][1], P01 = Pp[1][1 + o2], P11 = Pp[1 + o1][1 + o2];
#pragma unroll
      for (int q1 = 0; q1 < NQ1; ++q1) {
        const double pc1 = D1 ? 1.0 : (s1 == 0 ? kGX[q1] : 1.0 - kGX[q1]);
        const double po1 = 1.0 - pc1;
        const double w1 = D1 ? 1.0 : kGW[q1] * h1;
#pragma unroll
        for (int q2 = 0; q2 < NQ2; ++q2) {
          const double pc2 = D2 ? 1.0 : (s2 == 0 ? kGX[q2] : 1.0 - kGX[q2]);
          const double po2 = 1.0 - pc2;
          const double w = w1 * (D2 ? 1.0 : kGW[q2] * h2);
          const double phiI = pc1 * pc2;
          const double Th = phiI * T00 + po1 * pc2 * T10 + pc1 * po2 * T01 + po1 * po2 * T11;
          if (MODE == MODE_RES) {
            acc += w * g_rad_conv(g, Th) * phiI;
          } else if (DIAG) {
            acc += w * dg_rad_conv(g, Th) * phiI * phiI;
          } else {
            const double Ph = phiI * P00 + po1 * pc2 * P10 + pc1 * po2 * P01 + po1 * po2 * P11;
            acc += w * dg_rad_conv(g, Th) * phiI * Ph;
          }
        }
      }
    }
  }
  return g.dt * acc;
}

// local node index -> (i, j, k); 32-bit unsigned division whenever the local
// grid fits (64-bit division is a long software sequence: k_cg_diag spent most
// of its 63 us at C4 in it)
__device__ __forceinline__ void decode_node(int64_t n, const CgGrid& g, int& i, int& j, int& k) {
  if ((int64_t)g.n0 * g.n1 * g.n2 < (int64_t)0x7fffffff) {
    const uint32_t u = (uint32_t)n, n0 = (uint32_t)g.n0, n1 = (uint32_t)g.n1;
    const uint32_t q = u / n0;
    const uint32_t kk = q / n1;
    i = (int)(u - q * n0);
    j = (int)(q - kk * n1);
    k = (int)kk;
  } else {
    i = (int)(n % g.n0);
    j = (int)((n / g.n0) % g.n1);
    k = (int)(n / ((int64_t)g.n0 * g.n1));
  }
}

// Index maps along one axis, in closed form so no gathered address depends on
// a table load (the weights still come from the tables, independently): the
// coarse nodes are the even fine nodes and, for an odd cell count, the last
// one (fn - 1).
__device__ __forceinline__ void pmap(const MgXfer& x, int a, int i, int& c0, int& c1) {
  if (!x.coarse[a]) {
    c0 = c1 = i;
  } else if (!(i & 1)) {
    c0 = c1 = i >> 1;
  } else if (i == x.fn[a] - 1) {
    c0 = c1 = (i + 1) >> 1;
  } else {
    c0 = (i - 1) >> 1;
    c1 = (i + 1) >> 1;
  }
}
// the fine centre of coarse node I and its two neighbours (clamped to the centre
// where absent; their restriction weights are 0 there)
__device__ __forceinline__ void rmap(const MgXfer& x, int a, int I, int& f0, int& f1, int& f2) {
  if (!x.coarse[a]) {
    f0 = f1 = f2 = I;
    return;
  }
  const int nf = x.fn[a];
  f1 = (I == x.cn[a] - 1 && ((nf - 1) & 1)) ? nf - 1 : 2 * I;
  f0 = (f1 >= 1) ? f1 - 1 : f1;
  f2 = (f1 + 1 < nf) ? f1 + 1 : f1;
}

}  // namespace
}  // namespace tv
