// CG1 (Q1 quadrilateral / hexahedral) operators on UNSTRUCTURED meshes, gfx950:
// the element-local path for meshes that are not tensor-product grids (gmsh
// .msh input, distorted cells).
//
// Replaces, for such meshes, the FFCx cell kernel of F dx and its Jacobian
// (ThermoViscoProblem.py:295-300, ufl.derivative at :331) and the exterior-facet
// kernels of the Robin terms (:302-304), with the dolfinx assembly loops around
// them [3P]: gather the cell's vertex coordinates and dofs, evaluate the
// isoparametric element integral, scatter-add into the global vector.
//
// * One thread per cell: 2^d vertex ids (int32, [l][cell] layout: coalesced),
//   their coordinates and values gathered; the element integral with 3-point
//   Gauss per direction and the isoparametric Jacobian at every point (the
//   oracle's rule, oracle/tv_oracle.py HeatForm, so the two agree to rounding
//   on distorted cells); the 2^d results are added into the output vector.
// * Scatter without atomics: the cells are sorted into colours (no two cells of
//   a colour share a vertex, greedy colouring at context creation) and each
//   colour is one launch, so every add is a plain read-modify-write with no
//   conflict and the summation order is fixed (bitwise reproducible).
// * Robin facets: one thread per boundary facet (3-point Gauss per tangential
//   direction, surface measure |det J| |J^-T e_n| as the oracle), coloured the
//   same way.
// Algorithmic bytes of J x: 8 N (x) + 8 N (y) + 32 per cell
// (vertex ids) + 24 per vertex (coordinates) = ~72 B per cell on a hex mesh.
#include <algorithm>
#include <cstdio>
#include <vector>

#include "tv_device.h"

namespace tv {
namespace {

enum { UM_RES = 0, UM_JAC = 1, UM_DIAG = 2 };

__device__ constexpr double kUX[3] = {0.11270166537925831148, 0.5, 0.88729833462074168852};
__device__ constexpr double kUW[3] = {5.0 / 18.0, 8.0 / 18.0, 5.0 / 18.0};

__device__ __forceinline__ double um_g(const UmGrid& g, double T) {
  const double T2 = T * T;
  return g.a_rad * (T2 * T2 - g.T_amb4) + g.a_conv * (T - g.T_amb);
}
__device__ __forceinline__ double um_dg(const UmGrid& g, double T) { return g.a_rad * 4.0 * (T * T * T) + g.a_conv; }

// Q1 basis and reference gradients at xi (tensor order l = a + 2b + 4c)
template <int D>
__device__ __forceinline__ void q1(const double (&xi)[3], double (&phi)[1 << D], double (&dphi)[1 << D][D]) {
#pragma unroll
  for (int l = 0; l < (1 << D); ++l) {
    double f[3], df[3];
#pragma unroll
    for (int a = 0; a < D; ++a) {
      const int b = (l >> a) & 1;
      f[a] = b ? xi[a] : 1.0 - xi[a];
      df[a] = b ? 1.0 : -1.0;
    }
    double p = 1.0;
#pragma unroll
    for (int a = 0; a < D; ++a) p *= f[a];
    phi[l] = p;
#pragma unroll
    for (int a = 0; a < D; ++a) {
      double q = df[a];
#pragma unroll
      for (int e = 0; e < D; ++e)
        if (e != a) q *= f[e];
      dphi[l][a] = q;
    }
  }
}

// inverse and determinant of a D x D matrix
template <int D>
__device__ __forceinline__ double inv_det(const double (&J)[D][D], double (&Ji)[D][D]) {
  if constexpr (D == 2) {
    const double det = J[0][0] * J[1][1] - J[0][1] * J[1][0];
    const double id = 1.0 / det;
    Ji[0][0] = J[1][1] * id;
    Ji[0][1] = -J[0][1] * id;
    Ji[1][0] = -J[1][0] * id;
    Ji[1][1] = J[0][0] * id;
    return det;
  } else {
    double c[3][3];
    c[0][0] = J[1][1] * J[2][2] - J[1][2] * J[2][1];
    c[0][1] = J[0][2] * J[2][1] - J[0][1] * J[2][2];
    c[0][2] = J[0][1] * J[1][2] - J[0][2] * J[1][1];
    c[1][0] = J[1][2] * J[2][0] - J[1][0] * J[2][2];
    c[1][1] = J[0][0] * J[2][2] - J[0][2] * J[2][0];
    c[1][2] = J[0][2] * J[1][0] - J[0][0] * J[1][2];
    c[2][0] = J[1][0] * J[2][1] - J[1][1] * J[2][0];
    c[2][1] = J[0][1] * J[2][0] - J[0][0] * J[2][1];
    c[2][2] = J[0][0] * J[1][1] - J[0][1] * J[1][0];
    const double det = J[0][0] * c[0][0] + J[0][1] * c[1][0] + J[0][2] * c[2][0];
    const double id = 1.0 / det;
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) Ji[a][b] = c[a][b] * id;
    return det;
  }
}

// cell term of one colour: out[v] += element vector (RES: F dx part, JAC: J x,
// DIAG: diag J) -- ThermoViscoProblem.py:295-300 and its derivative
template <int D, int MODE>
__global__ __launch_bounds__(kBlock) void k_um_cells(UmGrid g, const double* __restrict__ u,
                                                     const double* __restrict__ up, double* __restrict__ out,
                                                     int64_t c0, int64_t c1) {
  constexpr int NL = 1 << D;
  const int64_t e = c0 + blockIdx.x * (int64_t)kBlock + threadIdx.x;
  if (e >= c1) return;
  int nd[NL];
  double X[NL][D], val[NL], mv[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    nd[l] = g.cell[(int64_t)l * g.nc + e];
#pragma unroll
    for (int a = 0; a < D; ++a) X[l][a] = g.X[a][nd[l]];
    val[l] = (MODE == UM_DIAG) ? 0.0 : u[nd[l]];
    mv[l] = (MODE == UM_RES) ? val[l] - up[nd[l]] : val[l];
  }
  double y[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) y[l] = 0.0;
  constexpr int NQ = (D == 2) ? 9 : 27;
#pragma unroll 1
  for (int q = 0; q < NQ; ++q) {
    const int qi[3] = {q % 3, (q / 3) % 3, q / 9};
    double xi[3] = {0.0, 0.0, 0.0}, w = 1.0;
#pragma unroll
    for (int a = 0; a < D; ++a) {
      xi[a] = kUX[qi[a]];
      w *= kUW[qi[a]];
    }
    double phi[NL], dphi[NL][D];
    q1<D>(xi, phi, dphi);
    double J[D][D];
#pragma unroll
    for (int a = 0; a < D; ++a)
#pragma unroll
      for (int b = 0; b < D; ++b) {
        double s = 0.0;
#pragma unroll
        for (int l = 0; l < NL; ++l) s += X[l][a] * dphi[l][b];
        J[a][b] = s;
      }
    double Ji[D][D];
    const double wd = w * fabs(inv_det<D>(J, Ji));
    // physical gradients: grad phi_l = J^-T dphi_l
    double gp[NL][D];
#pragma unroll
    for (int l = 0; l < NL; ++l)
#pragma unroll
      for (int a = 0; a < D; ++a) {
        double s = 0.0;
#pragma unroll
        for (int b = 0; b < D; ++b) s += Ji[b][a] * dphi[l][b];
        gp[l][a] = s;
      }
    if (MODE == UM_DIAG) {
#pragma unroll
      for (int l = 0; l < NL; ++l) {
        double gg = 0.0;
#pragma unroll
        for (int a = 0; a < D; ++a) gg += gp[l][a] * gp[l][a];
        y[l] += wd * (phi[l] * phi[l] + g.dt_alpha * gg);
      }
    } else {
      double mq = 0.0, gu[D];
#pragma unroll
      for (int a = 0; a < D; ++a) gu[a] = 0.0;
#pragma unroll
      for (int l = 0; l < NL; ++l) {
        mq += phi[l] * mv[l];
#pragma unroll
        for (int a = 0; a < D; ++a) gu[a] += gp[l][a] * val[l];
      }
      if (MODE == UM_RES) mq -= g.dt_f;
#pragma unroll
      for (int l = 0; l < NL; ++l) {
        double gg = 0.0;
#pragma unroll
        for (int a = 0; a < D; ++a) gg += gp[l][a] * gu[a];
        y[l] += wd * (phi[l] * mq + g.dt_alpha * gg);
      }
    }
  }
#pragma unroll
  for (int l = 0; l < NL; ++l) out[nd[l]] += y[l];
}

// Robin facets of one colour (ThermoViscoProblem.py:302-304 and derivative)
template <int D, int MODE>
__global__ __launch_bounds__(kBlock) void k_um_facets(UmGrid g, const double* __restrict__ T,
                                                      const double* __restrict__ x, double* __restrict__ out,
                                                      int64_t f0, int64_t f1) {
  constexpr int NL = 1 << D;
  const int64_t f = f0 + blockIdx.x * (int64_t)kBlock + threadIdx.x;
  if (f >= f1) return;
  const int64_t e = g.fcell[f];
  const int lf = g.flf[f];
  const int ax = lf >> 1, side = lf & 1;
  int nd[NL];
  double X[NL][D], Tv[NL], xv[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    nd[l] = g.cell[(int64_t)l * g.nc + e];
#pragma unroll
    for (int a = 0; a < D; ++a) X[l][a] = g.X[a][nd[l]];
    Tv[l] = T[nd[l]];
    xv[l] = (MODE == UM_JAC) ? x[nd[l]] : 0.0;
  }
  double y[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) y[l] = 0.0;
  constexpr int NQ = (D == 2) ? 3 : 9;
#pragma unroll 1
  for (int q = 0; q < NQ; ++q) {
    double xi[3] = {0.0, 0.0, 0.0}, w = 1.0;
    int t = 0;
#pragma unroll
    for (int a = 0; a < D; ++a) {
      if (a == ax) {
        xi[a] = (double)side;
        continue;
      }
      const int qi = (t == 0) ? (q % 3) : (q / 3);
      xi[a] = kUX[qi];
      w *= kUW[qi];
      ++t;
    }
    double phi[NL], dphi[NL][D];
    q1<D>(xi, phi, dphi);
    double J[D][D];
#pragma unroll
    for (int a = 0; a < D; ++a)
#pragma unroll
      for (int b = 0; b < D; ++b) {
        double s = 0.0;
#pragma unroll
        for (int l = 0; l < NL; ++l) s += X[l][a] * dphi[l][b];
        J[a][b] = s;
      }
    double Ji[D][D];
    const double det = fabs(inv_det<D>(J, Ji));
    double gn = 0.0;  // |row ax of J^-1| = |grad xi_ax|
#pragma unroll
    for (int b = 0; b < D; ++b) gn += Ji[ax][b] * Ji[ax][b];
    const double wm = w * det * sqrt(gn);
    double Tq = 0.0, xq = 0.0;
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      Tq += phi[l] * Tv[l];
      xq += phi[l] * xv[l];
    }
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      double v;
      if (MODE == UM_RES) v = um_g(g, Tq) * phi[l];
      else if (MODE == UM_JAC) v = um_dg(g, Tq) * xq * phi[l];
      else v = um_dg(g, Tq) * phi[l] * phi[l];
      y[l] += wm * v;
    }
  }
#pragma unroll
  for (int l = 0; l < NL; ++l)
    if (((l >> ax) & 1) == side) out[nd[l]] += g.dt * y[l];
}

__global__ __launch_bounds__(kBlock) void k_um_zero(double* __restrict__ x, int64_t n) {
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) x[t] = 0.0;
}
__global__ __launch_bounds__(kBlock) void k_um_invert(double* __restrict__ d, int64_t n) {
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) d[t] = 1.0 / d[t];
}

// PETSc KSPCG "p <- z + (beta / betaold) p" (p = z at iteration 0) into the
// buffer of this iteration's parity (the convention of k_pcg_update)
__global__ __launch_bounds__(kBlock) void k_um_pvec(int64_t n, const PcgState* __restrict__ st,
                                                    const double* __restrict__ z, double* pA, double* pB,
                                                    int it_host) {
  if (st->done) return;
  const bool first = it_host == 0;
  const double b = first ? 0.0 : st->beta / st->betaold;
  double* p = (it_host & 1) ? pB : pA;
  const double* po = (it_host & 1) ? pA : pB;
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock)
    p[t] = first ? z[t] : z[t] + b * po[t];
}

// partial records of p.w (width 1, fixed order)
__global__ __launch_bounds__(kBlock) void k_um_dot(int64_t n, const PcgState* __restrict__ st, const double* pA,
                                                   const double* pB, const double* __restrict__ w,
                                                   double* __restrict__ partials, int it_host) {
  __shared__ double red[kBlock / kWave];
  if (st->done) return;
  const double* p = (it_host & 1) ? pB : pA;
  double acc = 0.0;
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock)
    acc += p[t] * w[t];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) store_partial(&partials[blockIdx.x], (red[0] + red[1]) + (red[2] + red[3]));
}

int blocks_of(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + kBlock - 1) / kBlock, 1 << 20)); }
int vblocks(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + kBlock - 1) / kBlock, 1024)); }

template <int MODE>
void apply(const UmGrid& g, const double* T, const double* u, const double* up, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_um_zero, dim3(vblocks(g.nv)), dim3(kBlock), 0, s, out, g.nv);
  for (int k = 0; k < g.ncolor; ++k) {
    const int64_t c0 = g.color_off[k], c1 = g.color_off[k + 1];
    if (c1 <= c0) continue;
    if (g.dim == 2)
      hipLaunchKernelGGL((k_um_cells<2, MODE>), dim3(blocks_of(c1 - c0)), dim3(kBlock), 0, s, g, u, up, out, c0, c1);
    else
      hipLaunchKernelGGL((k_um_cells<3, MODE>), dim3(blocks_of(c1 - c0)), dim3(kBlock), 0, s, g, u, up, out, c0, c1);
  }
  for (int k = 0; k < g.nfcolor; ++k) {
    const int64_t f0 = g.fcolor_off[k], f1 = g.fcolor_off[k + 1];
    if (f1 <= f0) continue;
    if (g.dim == 2)
      hipLaunchKernelGGL((k_um_facets<2, MODE>), dim3(blocks_of(f1 - f0)), dim3(kBlock), 0, s, g, T, u, out, f0, f1);
    else
      hipLaunchKernelGGL((k_um_facets<3, MODE>), dim3(blocks_of(f1 - f0)), dim3(kBlock), 0, s, g, T, u, out, f0, f1);
  }
}

}  // namespace

void launch_um_residual(const UmGrid& g, const double* T, const double* Tp, double* F, hipStream_t s) {
  apply<UM_RES>(g, T, T, Tp, F, s);
}

void launch_um_japply(const UmGrid& g, const double* T, const double* x, double* y, hipStream_t s) {
  apply<UM_JAC>(g, T, x, nullptr, y, s);
}

void launch_um_diag(const UmGrid& g, const double* T, double* d, int invert, hipStream_t s) {
  apply<UM_DIAG>(g, T, nullptr, nullptr, d, s);
  if (invert) hipLaunchKernelGGL(k_um_invert, dim3(vblocks(g.nv)), dim3(kBlock), 0, s, d, g.nv);
}

int launch_um_japply_fused(const UmGrid& g, const double* T, const double* z, double* pA, double* pB, double* w,
                           const PcgState* st, double* partials, int it_host, hipStream_t s) {
  hipLaunchKernelGGL(k_um_pvec, dim3(vblocks(g.nv)), dim3(kBlock), 0, s, g.nv, st, z, pA, pB, it_host);
  apply<UM_JAC>(g, T, (it_host & 1) ? pB : pA, nullptr, w, s);
  const int nb = vblocks(g.nv);
  hipLaunchKernelGGL(k_um_dot, dim3(nb), dim3(kBlock), 0, s, g.nv, st, pA, pB, w, partials, it_host);
  return nb;
}

// ---- host: boundary facets and colouring ------------------------------------------
static int greedy_colour(const std::vector<std::vector<int64_t>>& items, int64_t nv, std::vector<int>& colour) {
  std::vector<uint64_t> used((size_t)nv, 0);
  colour.assign(items.size(), 0);
  int nc = 0;
  for (size_t e = 0; e < items.size(); ++e) {
    uint64_t m = 0;
    for (int64_t v : items[e]) m |= used[(size_t)v];
    int c = 0;
    while (c < 64 && ((m >> c) & 1)) ++c;
    if (c == 64) return -1;
    colour[e] = c;
    nc = std::max(nc, c + 1);
    for (int64_t v : items[e]) used[(size_t)v] |= (uint64_t)1 << c;
  }
  return nc;
}

int um_build(int dim, int64_t nv, int64_t nc, const int64_t* cells, UmHost& out, std::string& err) {
  const int nl = 1 << dim;
  // boundary facets: local facets whose sorted vertex set occurs once
  struct F {
    int64_t v[4];
    int64_t cell;
    int lf;
  };
  const int nfv = nl / 2;
  std::vector<F> fs;
  fs.reserve((size_t)nc * 2 * dim);
  for (int64_t e = 0; e < nc; ++e)
    for (int lf = 0; lf < 2 * dim; ++lf) {
      F f{{-1, -1, -1, -1}, e, lf};
      int k = 0;
      for (int l = 0; l < nl; ++l)
        if (((l >> (lf >> 1)) & 1) == (lf & 1)) f.v[k++] = cells[e * nl + l];
      std::sort(f.v, f.v + nfv);
      fs.push_back(f);
    }
  auto key_less = [&](const F& a, const F& b) {
    for (int k = 0; k < nfv; ++k)
      if (a.v[k] != b.v[k]) return a.v[k] < b.v[k];
    return false;
  };
  auto key_eq = [&](const F& a, const F& b) {
    for (int k = 0; k < nfv; ++k)
      if (a.v[k] != b.v[k]) return false;
    return true;
  };
  std::sort(fs.begin(), fs.end(), [&](const F& a, const F& b) {
    if (key_less(a, b)) return true;
    if (key_less(b, a)) return false;
    return a.cell < b.cell;
  });
  std::vector<std::pair<int64_t, int>> bf;
  for (size_t i = 0; i < fs.size();) {
    size_t j = i + 1;
    while (j < fs.size() && key_eq(fs[i], fs[j])) ++j;
    if (j - i == 1) bf.emplace_back(fs[i].cell, fs[i].lf);
    else if (j - i > 2) {
      err = "non-manifold mesh: a facet shared by more than two cells";
      return -1;
    }
    i = j;
  }
  std::sort(bf.begin(), bf.end());
  // colour the cells and the boundary facets
  std::vector<std::vector<int64_t>> items((size_t)nc);
  for (int64_t e = 0; e < nc; ++e) items[e].assign(cells + e * nl, cells + (e + 1) * nl);
  std::vector<int> col;
  const int ncol = greedy_colour(items, nv, col);
  if (ncol < 0) {
    err = "more than 64 colours needed";
    return -1;
  }
  std::vector<std::vector<int64_t>> fitems(bf.size());
  for (size_t f = 0; f < bf.size(); ++f) {
    const int64_t e = bf[f].first;
    const int lf = bf[f].second;
    for (int l = 0; l < nl; ++l)
      if (((l >> (lf >> 1)) & 1) == (lf & 1)) fitems[f].push_back(cells[e * nl + l]);
  }
  std::vector<int> fcol;
  const int nfcol = greedy_colour(fitems, nv, fcol);
  if (nfcol < 0) {
    err = "more than 64 facet colours needed";
    return -1;
  }
  // cells sorted by colour (stable: cell order within a colour); [l][cell] layout
  std::vector<int64_t> order((size_t)nc);
  for (int64_t e = 0; e < nc; ++e) order[e] = e;
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return col[a] < col[b]; });
  std::vector<int64_t> pos((size_t)nc);
  for (int64_t k = 0; k < nc; ++k) pos[order[k]] = k;
  out.cell.assign((size_t)nl * nc, 0);
  for (int64_t k = 0; k < nc; ++k)
    for (int l = 0; l < nl; ++l) out.cell[(size_t)l * nc + k] = (int)cells[order[k] * nl + l];
  out.color_off.assign(ncol + 1, 0);
  for (int64_t e = 0; e < nc; ++e) out.color_off[col[e] + 1]++;
  for (int k = 0; k < ncol; ++k) out.color_off[k + 1] += out.color_off[k];
  std::vector<int64_t> forder(bf.size());
  for (size_t f = 0; f < bf.size(); ++f) forder[f] = (int64_t)f;
  std::stable_sort(forder.begin(), forder.end(), [&](int64_t a, int64_t b) { return fcol[a] < fcol[b]; });
  out.fcell.resize(bf.size());
  out.flf.resize(bf.size());
  for (size_t k = 0; k < bf.size(); ++k) {
    out.fcell[k] = (int)pos[bf[forder[k]].first];  // the cell's position in the coloured order
    out.flf[k] = (signed char)bf[forder[k]].second;
  }
  out.fcolor_off.assign(nfcol + 1, 0);
  for (size_t f = 0; f < bf.size(); ++f) out.fcolor_off[fcol[f] + 1]++;
  for (int k = 0; k < nfcol; ++k) out.fcolor_off[k + 1] += out.fcolor_off[k];
  return 0;
}


// ---- host: recursive coordinate bisection of the cells ----------------------------
// Splits the cell set along the axis of largest centroid extent so that the two
// halves hold cells in proportion to the part counts they receive (any number of
// parts, not only powers of two).  Deterministic: ties broken by cell index.
// Replaces the graph partitioner dolfinx calls when a mesh is distributed
// (create_mesh with the default partitioner, gmshio.read_from_msh at
// ThermoViscoProblem.py:27-28).
static void rcb_split(const std::vector<double>& cen, std::vector<int64_t>& idx, int64_t lo, int64_t hi, int p0,
                      int np, int* part) {
  if (np == 1) {
    for (int64_t k = lo; k < hi; ++k) part[idx[(size_t)k]] = p0;
    return;
  }
  double mn[3] = {1e300, 1e300, 1e300}, mx[3] = {-1e300, -1e300, -1e300};
  for (int64_t k = lo; k < hi; ++k)
    for (int a = 0; a < 3; ++a) {
      const double v = cen[3 * (size_t)idx[(size_t)k] + a];
      mn[a] = std::min(mn[a], v);
      mx[a] = std::max(mx[a], v);
    }
  int ax = 0;
  for (int a = 1; a < 3; ++a)
    if (mx[a] - mn[a] > mx[ax] - mn[ax]) ax = a;
  const int nl = np / 2;
  const int64_t mid = lo + (int64_t)((double)(hi - lo) * nl / np + 0.5);
  auto less = [&](int64_t x, int64_t y) {
    const double vx = cen[3 * (size_t)x + ax], vy = cen[3 * (size_t)y + ax];
    return vx < vy || (vx == vy && x < y);
  };
  std::nth_element(idx.begin() + lo, idx.begin() + mid, idx.begin() + hi, less);
  rcb_split(cen, idx, lo, mid, p0, nl, part);
  rcb_split(cen, idx, mid, hi, p0 + nl, np - nl, part);
}

int um_rcb(int dim, int64_t nv, const double* xyz, int64_t nc, const int64_t* cells, int n_parts, int* part,
           std::string& err) {
  if (n_parts < 1 || n_parts > nc) {
    err = "n_parts must be in [1, n_cells]";
    return 1;
  }
  const int nl = 1 << dim;
  std::vector<double> cen((size_t)3 * nc, 0.0);
  for (int64_t e = 0; e < nc; ++e)
    for (int l = 0; l < nl; ++l) {
      const int64_t v = cells[(size_t)e * nl + l];
      if (v < 0 || v >= nv) {
        err = "cell vertex index out of range";
        return 1;
      }
      for (int a = 0; a < 3; ++a) cen[3 * (size_t)e + a] += xyz[3 * (size_t)v + a] / nl;
    }
  std::vector<int64_t> idx((size_t)nc);
  for (int64_t e = 0; e < nc; ++e) idx[(size_t)e] = e;
  rcb_split(cen, idx, 0, nc, 0, n_parts, part);
  return 0;
}

}  // namespace tv
