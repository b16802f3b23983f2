// Smoothed-aggregation algebraic multigrid (options.preconditioner = TV_PC_AMG)
// for the unstructured meshes: host setup of the hierarchy and the V-cycle.
//
// The reference preconditions its CG with PETSc's PCGAMG (ThermoViscoProblem.py:
// 343-346), a smoothed-aggregation AMG built from the assembled matrix; the box
// meshes use the geometric hierarchy of tv_mgsolve.cpp instead.  Here, for
// general hexahedra / quadrilaterals:
//   * the hierarchy is built ONCE, from the T-independent cell operator
//     V = M + dt alpha K (the SELL-64 matrix tv_um.hip assembles at creation);
//     the Robin term of J(T) enters the fine level only (its diagonal in the
//     smoother, its product in the Krylov matvec), so B is a fixed SPD
//     operator per Newton iteration and CG stays CG;
//   * aggregation: greedy, every off-diagonal nonzero strong (PCGAMG's default
//     threshold 0): (1) a node whose neighbours are all free seeds an aggregate
//     of itself and its neighbours, (2) the remaining free nodes join the
//     aggregate of their first aggregated neighbour, (3) leftovers seed
//     aggregates of their free neighbours;
//   * tentative prolongation: piecewise constant (the constant near-null
//     space of the heat operator); smoothed P = (I - 4/3 / lambda D^-1 A) P0,
//     lambda = lambda_max(D^-1 A) by power iteration, stored in float32
//     (SELL-64, like R = P^T: the transfers are the cycle's largest
//     streams); Galerkin A_c = P^T A P in double from the rounded P;
//     until <= kAmgCoarseRows rows (or the options.mg_levels depth);
//   * structured topology (vertex i + N0 (j + N1 k), the box's cells, any
//     coordinates: tv_um.hip's half-stencil meshes): the tentative-and-smoothed
//     P is replaced by the geometric one of the index space -- every other
//     vertex kept along each axis (plus the last when the cell count is odd),
//     the others linearly interpolated with weights 1/2 (exact in float32) --
//     and every coarse level is again a structured grid; A_c = P^T A P as
//     above.  Numpy model of the distorted plate (120 x 120 x 14 cells, random
//     right-hand side): smoothed aggregation 13 Krylov iterations, this
//     hierarchy with the same additive cycle 11, and 3.4 instead of ~20 stored
//     transfer entries per fine row;
//   * cycle: level 0 ADDITIVE -- z = omega0 D^-1 r + P_0 V_1(P_0^T r) -- so the
//     preconditioner never applies the fine operator (a fine J x streams
//     ~330 B per row on these meshes; the Krylov matvec is the only one per
//     iteration); levels >= 1 multiplicative V(1,1) with damped Jacobi
//     (omega = 2 / (1.1 lambda_max(D^-1 A_l))), one Jacobi step on the
//     coarsest level.  Measured in a numpy model of the distorted plate
//     (544K vertices, the Newton right-hand side): Jacobi-PCG 35 iterations,
//     this cycle 12, a multiplicative V(1,1) 11 (at three fine J x per
//     iteration instead of one), unsmoothed aggregation 16.
#include <numeric>
#include <thread>

#include "tv_ctx.h"

namespace tv {
namespace {

constexpr int64_t kAmgCoarseRows = 2000;
constexpr int64_t kAmgSortWindow = 4096;  // rows per length-sorting window of the transfers' SELL layout

struct Csr {
  int64_t n = 0, m = 0;  // rows, columns
  std::vector<int64_t> ptr;
  std::vector<int> col;
  std::vector<double> val;
};

int n_workers() {
  const unsigned h = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(16u, h ? h : 1u));
}

// f(t, r0, r1) on contiguous row ranges, one per worker thread
template <class F>
void par_ranges(int64_t n, F f) {
  const int nt = (int)std::min<int64_t>(n_workers(), std::max<int64_t>(1, n / 4096));
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) th.emplace_back([&, t]() { f(t, n * t / nt, n * (t + 1) / nt); });
  for (auto& x : th) x.join();
}

void spmv(const Csr& A, const std::vector<double>& x, std::vector<double>& y) {
  par_ranges(A.n, [&](int, int64_t r0, int64_t r1) {
    for (int64_t r = r0; r < r1; ++r) {
      double s = 0.0;
      for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) s += A.val[k] * x[A.col[k]];
      y[r] = s;
    }
  });
}

std::vector<double> diag_inv(const Csr& A) {
  std::vector<double> d((size_t)A.n, 0.0);
  for (int64_t r = 0; r < A.n; ++r)
    for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k)
      if (A.col[k] == (int)r) d[r] = 1.0 / A.val[k];
  return d;
}

// largest eigenvalue of the symmetric tridiagonal matrix (a, b) by bisection
// on the Sturm sequence count (full double precision, 200 halvings at most)
double tridiag_max_eig(const std::vector<double>& a, const std::vector<double>& b) {
  const size_t k = a.size();
  double lo = a[0], hi = a[0];
  for (size_t i = 0; i < k; ++i) {
    const double r = (i > 0 ? std::fabs(b[i - 1]) : 0.0) + (i + 1 < k ? std::fabs(b[i]) : 0.0);
    lo = std::min(lo, a[i] - r);
    hi = std::max(hi, a[i] + r);
  }
  auto below = [&](double x) {  // eigenvalues < x
    size_t cnt = 0;
    double d = 1.0;
    for (size_t i = 0; i < k; ++i) {
      d = a[i] - x - (i > 0 ? b[i - 1] * b[i - 1] / d : 0.0);
      if (d == 0.0) d = -1e-300;
      if (d < 0.0) ++cnt;
    }
    return cnt;
  };
  for (int it = 0; it < 200 && hi - lo > 1e-15 * std::max(std::fabs(lo), std::fabs(hi)); ++it) {
    const double mid = 0.5 * (lo + hi);
    if (below(mid) == k) hi = mid; else lo = mid;
  }
  return hi;
}

// lambda_max(D^-1 A) (A SPD): the largest Ritz value of `its` Lanczos steps on
// D^-1/2 A D^-1/2 from a fixed-seed start vector (reproducible).  The extreme
// Ritz value converges much faster than a power iteration (whose estimate
// stalls below lambda_max when the top eigenvalues cluster; the smoothing
// weights 2 / (1.1 lambda) must not exceed 2 / lambda_max) -- PETSc's GAMG
// estimates it by Krylov iterations too (esteig).
double lam_max(const Csr& A, const std::vector<double>& dinv, int its) {
  const size_t n = (size_t)A.n;
  std::vector<double> q(n), qp(n, 0.0), w(n), t(n), sd(n);
  for (size_t r = 0; r < n; ++r) sd[r] = std::sqrt(dinv[r]);
  uint64_t st = 0x2545F4914F6CDD1Dull;
  double nv = 0.0;
  for (auto& e : q) {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    e = 0.5 + (double)(st >> 11) * (1.0 / 9007199254740992.0);
    nv += e * e;
  }
  nv = std::sqrt(nv);
  for (auto& e : q) e /= nv;
  std::vector<double> al, be;
  double beta = 0.0;
  for (int j = 0; j < its; ++j) {
    for (size_t r = 0; r < n; ++r) t[r] = sd[r] * q[r];
    spmv(A, t, w);
    double alpha = 0.0;
    for (size_t r = 0; r < n; ++r) {
      w[r] = sd[r] * w[r] - beta * qp[r];
      alpha += w[r] * q[r];
    }
    double bn = 0.0;
    for (size_t r = 0; r < n; ++r) {
      w[r] -= alpha * q[r];
      bn += w[r] * w[r];
    }
    al.push_back(alpha);
    beta = std::sqrt(bn);
    if (j + 1 == its || !(beta > 0.0)) break;
    be.push_back(beta);
    qp.swap(q);
    for (size_t r = 0; r < n; ++r) q[r] = w[r] / beta;
  }
  return tridiag_max_eig(al, be);
}

// greedy aggregation (see the header); returns the aggregate of every row
std::vector<int> aggregate(const Csr& A, int64_t& na) {
  std::vector<int> agg((size_t)A.n, -1);
  na = 0;
  for (int64_t i = 0; i < A.n; ++i) {  // pass 1: seeds with all neighbours free
    if (agg[i] >= 0) continue;
    bool free = true;
    for (int64_t k = A.ptr[i]; k < A.ptr[i + 1] && free; ++k) free = agg[A.col[k]] < 0;
    if (!free) continue;
    for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k) agg[A.col[k]] = (int)na;
    agg[i] = (int)na++;
  }
  std::vector<int> join((size_t)A.n, -1);
  for (int64_t i = 0; i < A.n; ++i) {  // pass 2: join the first aggregated neighbour
    if (agg[i] >= 0) continue;
    for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k)
      if (agg[A.col[k]] >= 0) {
        join[i] = agg[A.col[k]];
        break;
      }
  }
  for (int64_t i = 0; i < A.n; ++i)
    if (join[i] >= 0) agg[i] = join[i];
  for (int64_t i = 0; i < A.n; ++i) {  // pass 3: leftovers with their free neighbours
    if (agg[i] >= 0) continue;
    for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k)
      if (agg[A.col[k]] < 0) agg[A.col[k]] = (int)na;
    agg[i] = (int)na++;
  }
  return agg;
}

// P = (I - w D^-1 A) P0, P0 the aggregate indicator (columns sorted per row)
Csr smoothed_p(const Csr& A, const std::vector<double>& dinv, const std::vector<int>& agg, int64_t na, double w) {
  Csr P;
  P.n = A.n;
  P.m = na;
  std::vector<int64_t> cnt((size_t)A.n + 1, 0);
  std::vector<std::vector<int>> cols_t((size_t)n_workers());
  std::vector<std::vector<double>> vals_t((size_t)n_workers());
  std::vector<std::pair<int64_t, int64_t>> rng((size_t)n_workers(), {0, 0});
  par_ranges(A.n, [&](int t, int64_t r0, int64_t r1) {
    rng[t] = {r0, r1};
    std::vector<std::pair<int, double>> e;
    for (int64_t i = r0; i < r1; ++i) {
      e.clear();
      e.emplace_back(agg[i], 1.0);
      for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k) e.emplace_back(agg[A.col[k]], -w * dinv[i] * A.val[k]);
      std::stable_sort(e.begin(), e.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
      int64_t c0 = 0;
      for (size_t q = 0; q < e.size();) {  // merge equal aggregates (fixed order: deterministic sums)
        size_t u = q;
        double s = 0.0;
        while (u < e.size() && e[u].first == e[q].first) s += e[u++].second;
        cols_t[t].push_back(e[q].first);
        vals_t[t].push_back(s);
        ++c0;
        q = u;
      }
      cnt[i + 1] = c0;
    }
  });
  P.ptr.assign((size_t)A.n + 1, 0);
  for (int64_t i = 0; i < A.n; ++i) P.ptr[i + 1] = P.ptr[i] + cnt[i + 1];
  P.col.resize((size_t)P.ptr[A.n]);
  P.val.resize((size_t)P.ptr[A.n]);
  for (size_t t = 0; t < rng.size(); ++t) {
    if (rng[t].second <= rng[t].first) continue;
    std::copy(cols_t[t].begin(), cols_t[t].end(), P.col.begin() + P.ptr[rng[t].first]);
    std::copy(vals_t[t].begin(), vals_t[t].end(), P.val.begin() + P.ptr[rng[t].first]);
  }
  return P;
}

Csr transpose(const Csr& P) {
  Csr R;
  R.n = P.m;
  R.m = P.n;
  R.ptr.assign((size_t)R.n + 1, 0);
  for (int c : P.col) R.ptr[(size_t)c + 1]++;
  for (int64_t r = 0; r < R.n; ++r) R.ptr[r + 1] += R.ptr[r];
  R.col.resize(P.col.size());
  R.val.resize(P.val.size());
  std::vector<int64_t> fill(R.ptr.begin(), R.ptr.end() - 1);
  for (int64_t i = 0; i < P.n; ++i)  // rows in order: each R row's columns ascend
    for (int64_t k = P.ptr[i]; k < P.ptr[i + 1]; ++k) {
      const int64_t q = fill[P.col[k]]++;
      R.col[q] = (int)i;
      R.val[q] = P.val[k];
    }
  return R;
}

// C = A B (rows in parallel, a dense accumulator per worker; columns sorted)
Csr spgemm(const Csr& A, const Csr& B) {
  Csr C;
  C.n = A.n;
  C.m = B.m;
  const int nw = n_workers();
  std::vector<std::vector<int>> cols_t((size_t)nw);
  std::vector<std::vector<double>> vals_t((size_t)nw);
  std::vector<std::pair<int64_t, int64_t>> rng((size_t)nw, {0, 0});
  std::vector<int64_t> cnt((size_t)A.n + 1, 0);
  par_ranges(A.n, [&](int t, int64_t r0, int64_t r1) {
    rng[t] = {r0, r1};
    std::vector<double> acc((size_t)B.m, 0.0);
    std::vector<int> mark((size_t)B.m, -1), touched;
    for (int64_t i = r0; i < r1; ++i) {
      touched.clear();
      for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k) {
        const double a = A.val[k];
        const int j = A.col[k];
        for (int64_t q = B.ptr[j]; q < B.ptr[j + 1]; ++q) {
          const int c = B.col[q];
          if (mark[c] != (int)i) {
            mark[c] = (int)i;
            acc[c] = 0.0;
            touched.push_back(c);
          }
          acc[c] += a * B.val[q];
        }
      }
      std::sort(touched.begin(), touched.end());
      for (int c : touched) {
        cols_t[t].push_back(c);
        vals_t[t].push_back(acc[c]);
      }
      cnt[i + 1] = (int64_t)touched.size();
    }
  });
  C.ptr.assign((size_t)A.n + 1, 0);
  for (int64_t i = 0; i < A.n; ++i) C.ptr[i + 1] = C.ptr[i] + cnt[i + 1];
  C.col.resize((size_t)C.ptr[A.n]);
  C.val.resize((size_t)C.ptr[A.n]);
  for (size_t t = 0; t < rng.size(); ++t) {
    if (rng[t].second <= rng[t].first) continue;
    std::copy(cols_t[t].begin(), cols_t[t].end(), C.col.begin() + C.ptr[rng[t].first]);
    std::copy(vals_t[t].begin(), vals_t[t].end(), C.val.begin() + C.ptr[rng[t].first]);
  }
  return C;
}

template <class T>
int amg_alloc(Ctx* c, size_t n, T** out) {
  void* p = nullptr;
  HIPC(hipMalloc(&p, sizeof(T) * std::max<size_t>(1, n)));
  c->amg_bufs.push_back(p);
  *out = static_cast<T*>(p);
  return TV_OK;
}

template <class T>
int amg_upload(Ctx* c, const std::vector<T>& h, T** out) {
  if (int e = amg_alloc(c, h.size(), out)) return e;
  if (!h.empty()) HIPC(hipMemcpy(*out, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice));
  return TV_OK;
}

// CSR -> the device: SELL-64 (padding: value 0, column 0) or CSR (as is);
// values in float32 (the transfers) or double
int upload_mat(Ctx* c, const Csr& M, Sell& out, bool csr, bool fp32, int64_t sort_window, int64_t* stored) {
  const int64_t ns = (M.n + 63) / 64;
  std::vector<int64_t> soff;
  std::vector<int> cols;
  std::vector<double> vals;
  std::vector<int> perm;
  if (csr) {
    soff = M.ptr;
    cols = M.col;
    vals = M.val;
  } else {
    // sort_window > 0: rows ordered by decreasing length inside windows of that
    // many rows (stable), so each 64-row slice pads to a similar length
    perm.resize((size_t)M.n);
    std::iota(perm.begin(), perm.end(), 0);
    if (sort_window > 0)
      for (int64_t w0 = 0; w0 < M.n; w0 += sort_window) {
        const int64_t w1 = std::min(M.n, w0 + sort_window);
        std::stable_sort(perm.begin() + w0, perm.begin() + w1, [&](int a, int b) {
          return M.ptr[a + 1] - M.ptr[a] > M.ptr[b + 1] - M.ptr[b];
        });
      }
    auto len = [&](int64_t q) { return M.ptr[perm[q] + 1] - M.ptr[perm[q]]; };
    soff.assign((size_t)ns + 1, 0);
    for (int64_t s = 0; s < ns; ++s) {
      int64_t w = 0;
      for (int64_t q = s * 64; q < std::min(M.n, s * 64 + 64); ++q) w = std::max(w, len(q));
      soff[s + 1] = soff[s] + 64 * w;
    }
    cols.assign((size_t)soff[ns], 0);
    vals.assign((size_t)soff[ns], 0.0);
    for (int64_t q = 0; q < M.n; ++q) {
      const int64_t s = q >> 6, lane = q & 63, r = perm[q];
      for (int64_t k = M.ptr[r]; k < M.ptr[r + 1]; ++k) {
        const int64_t o = soff[s] + 64 * (k - M.ptr[r]) + lane;
        cols[o] = M.col[k];
        vals[o] = M.val[k];
      }
    }
  }
  if (stored) *stored = (int64_t)cols.size();
  int64_t* so;
  int* co;
  if (int e = amg_upload(c, soff, &so)) return e;
  if (int e = amg_upload(c, cols, &co)) return e;
  if (fp32) {
    std::vector<float> vf(vals.begin(), vals.end());
    float* va;
    if (int e = amg_upload(c, vf, &va)) return e;
    out.vals = va;
  } else {
    double* va;
    if (int e = amg_upload(c, vals, &va)) return e;
    out.vals = va;
  }
  out.perm = nullptr;
  if (!csr && sort_window > 0) {
    int* pd;
    if (int e = amg_upload(c, perm, &pd)) return e;
    out.perm = pd;
  }
  out.nrow = M.n;
  out.ncol = M.m;
  out.nslice = ns;
  out.soff = so;
  out.cols = co;
  out.csr = csr ? 1 : 0;
  out.fp32 = fp32 ? 1 : 0;
  return TV_OK;
}

// the fine SELL-64 operator back on the host as CSR (padding entries dropped)
int fine_csr(Ctx* c, Csr& A) {
  const Sell S = um_operator(c->umg);
  std::vector<int64_t> soff((size_t)S.nslice + 1);
  HIPC(hipMemcpy(soff.data(), S.soff, sizeof(int64_t) * soff.size(), hipMemcpyDeviceToHost));
  const int64_t nnz = soff[S.nslice];
  std::vector<int> cols((size_t)nnz);
  std::vector<double> vals((size_t)nnz);
  HIPC(hipMemcpy(cols.data(), S.cols, sizeof(int) * (size_t)nnz, hipMemcpyDeviceToHost));
  HIPC(hipMemcpy(vals.data(), S.vals, sizeof(double) * (size_t)nnz, hipMemcpyDeviceToHost));
  A.n = S.nrow;
  A.m = S.ncol;
  A.ptr.assign((size_t)A.n + 1, 0);
  for (int64_t r = 0; r < A.n; ++r) {
    const int64_t s = r >> 6, lane = r & 63, w = (soff[s + 1] - soff[s]) >> 6;
    int64_t k = 0;
    for (int64_t q = 0; q < w; ++q)
      if (vals[(size_t)(soff[s] + 64 * q + lane)] != 0.0) ++k;
    A.ptr[r + 1] = A.ptr[r] + k;
  }
  A.col.resize((size_t)A.ptr[A.n]);
  A.val.resize((size_t)A.ptr[A.n]);
  for (int64_t r = 0; r < A.n; ++r) {
    const int64_t s = r >> 6, lane = r & 63, w = (soff[s + 1] - soff[s]) >> 6;
    int64_t k = A.ptr[r];
    for (int64_t q = 0; q < w; ++q) {
      const size_t e = (size_t)(soff[s] + 64 * q + lane);
      if (vals[e] != 0.0) {
        A.col[k] = cols[e];
        A.val[k++] = vals[e];
      }
    }
  }
  return TV_OK;
}

// The geometric prolongation of a structured grid of n[0] x n[1] x n[2]
// vertices (vertex i + n0 (j + n1 k)) onto its index-space coarsening; the
// coarse grid's node counts in nc.  Per axis: fine node 2c is coarse node c, an
// odd fine node between two kept ones takes 1/2 of each, and the last node is
// kept when the cell count is odd.
Csr geometric_p(const int64_t (&n)[3], int64_t (&nc)[3]) {
  std::vector<int> ci[3][2];
  std::vector<double> cw[3][2];
  for (int a = 0; a < 3; ++a) {
    const int64_t m = n[a];
    std::vector<int> pos((size_t)m, -1);
    int64_t c = 0;
    for (int64_t i = 0; i < m; i += 2) pos[(size_t)i] = (int)c++;
    if (pos[(size_t)(m - 1)] < 0) pos[(size_t)(m - 1)] = (int)c++;
    nc[a] = c;
    for (int s = 0; s < 2; ++s) {
      ci[a][s].assign((size_t)m, -1);
      cw[a][s].assign((size_t)m, 0.0);
    }
    for (int64_t i = 0; i < m; ++i) {
      if (pos[(size_t)i] >= 0) {
        ci[a][0][(size_t)i] = pos[(size_t)i];
        cw[a][0][(size_t)i] = 1.0;
      } else {  // between two kept nodes (columns ascending)
        ci[a][0][(size_t)i] = pos[(size_t)(i - 1)];
        ci[a][1][(size_t)i] = pos[(size_t)(i + 1)];
        cw[a][0][(size_t)i] = cw[a][1][(size_t)i] = 0.5;
      }
    }
  }
  Csr P;
  P.n = n[0] * n[1] * n[2];
  P.m = nc[0] * nc[1] * nc[2];
  P.ptr.assign((size_t)P.n + 1, 0);
  for (int64_t k = 0, r = 0; k < n[2]; ++k)
    for (int64_t j = 0; j < n[1]; ++j)
      for (int64_t i = 0; i < n[0]; ++i, ++r) {
        int cnt = 1;
        for (int a = 0; a < 3; ++a) cnt *= (ci[a][1][(size_t)(a == 0 ? i : a == 1 ? j : k)] >= 0) ? 2 : 1;
        P.ptr[(size_t)r + 1] = P.ptr[(size_t)r] + cnt;
      }
  P.col.resize((size_t)P.ptr[(size_t)P.n]);
  P.val.resize(P.col.size());
  for (int64_t k = 0, r = 0; k < n[2]; ++k)
    for (int64_t j = 0; j < n[1]; ++j)
      for (int64_t i = 0; i < n[0]; ++i, ++r) {
        int64_t e = P.ptr[(size_t)r];
        for (int sk = 0; sk < 2; ++sk) {  // columns ascending: k slowest
          const int cK = ci[2][sk][(size_t)k];
          if (cK < 0) continue;
          for (int sj = 0; sj < 2; ++sj) {
            const int cJ = ci[1][sj][(size_t)j];
            if (cJ < 0) continue;
            for (int si = 0; si < 2; ++si) {
              const int cI = ci[0][si][(size_t)i];
              if (cI < 0) continue;
              P.col[(size_t)e] = (int)(cI + nc[0] * (cJ + nc[1] * (int64_t)cK));
              P.val[(size_t)e++] = cw[0][si][(size_t)i] * cw[1][sj][(size_t)j] * cw[2][sk][(size_t)k];
            }
          }
        }
      }
  return P;
}

// A (n = d0 d1 d2 rows of a structured grid, 27-point couplings) as the upper
// half stencil of tv_um.hip (slot q - 13 of row r: column r + o_q, q >= 13),
// uploaded into sg; false when A is not such an operator (a coupling beyond the
// 27 neighbours, or an axis too short to decode offsets) -- the level keeps SELL
bool half_stencil(Ctx* c, const Csr& A, const int64_t (&d)[3], UmGrid& sg) {
  if (d[0] < 3 || d[1] < 3 || d[2] < 2) return false;
  const int64_t n = A.n, s1 = d[0], s2 = d[0] * d[1];
  std::vector<double> X((size_t)14 * n, 0.0);
  for (int64_t r = 0; r < n; ++r) {
    const int64_t i = r % s1, j = (r / s1) % d[1], k = r / s2;
    for (int64_t e = A.ptr[r]; e < A.ptr[r + 1]; ++e) {
      const int64_t cc = A.col[e];
      const int64_t ci = cc % s1, cj = (cc / s1) % d[1], ck = cc / s2;
      const int64_t di = ci - i, dj = cj - j, dk = ck - k;
      if (di < -1 || di > 1 || dj < -1 || dj > 1 || dk < -1 || dk > 1) return false;
      const int q = (int)((di + 1) + 3 * (dj + 1) + 9 * (dk + 1));
      if (q >= 13) X[(size_t)(q - 13) * n + r] = A.val[e];
    }
  }
  double* dX = nullptr;
  if (amg_upload(c, X, &dX)) return false;
  sg = UmGrid{};
  sg.dim = 3;
  sg.nv = sg.nrow = n;
  sg.s1 = s1;
  sg.s2 = s2;
  sg.V14 = dX;
  sg.J14 = dX;
  return true;
}

}  // namespace

// builds the hierarchy below the fine level from the fine operator A.  One
// partition: A = the local operator.  Partitioned (amg_setup_part): A = the
// GLOBAL operator in the partition-major numbering, identical on every rank,
// and the level-0 transfer is cut to this rank's owned fine rows
// [row0, row0 + nrow) -- P_0 (owned fine rows x all level-1 aggregates) and
// R_0 = P_0^T; levels >= 1 are replicated on every rank (agglomerated).
// grid: the structured grid's vertex counts (geometric transfers, one
// partition) or nullptr (smoothed aggregation)
static int amg_build(Ctx* c, Csr A, int64_t row0, int64_t nrow, const int64_t* grid = nullptr) {
  const bool part = c->n_parts > 1;
  const int max_levels = c->O.mg_levels > 0 ? c->O.mg_levels : 12;
  int64_t dims[3] = {grid ? grid[0] : 0, grid ? grid[1] : 0, grid ? grid[2] : 0};
  while ((int)c->amg.size() + 1 < max_levels && A.n > kAmgCoarseRows) {
    int64_t na = 0;
    Csr P;
    int64_t fdims[3] = {dims[0], dims[1], dims[2]};
    if (grid) {
      int64_t cd[3];
      P = geometric_p(dims, cd);
      na = P.m;
      if (na * 10 > A.n * 7) break;  // the axes no longer coarsen
      for (int a = 0; a < 3; ++a) dims[a] = cd[a];
    } else {
      const std::vector<double> dinv = diag_inv(A);
      const std::vector<int> agg = aggregate(A, na);
      if (na < 1 || na * 10 > A.n * 7) break;  // coarsening stalled
      const double lam = lam_max(A, dinv, 20);
      P = smoothed_p(A, dinv, agg, na, 4.0 / (3.0 * lam));
    }
    // the transfers are stored in float32 (half the bytes of the V-cycle's
    // largest streams): round P first, so R = P^T and A_c = R (A P) are built
    // from the very values the device applies (the cycle stays symmetric)
    for (double& v : P.val) v = (double)(float)v;
    Csr R = transpose(P);
    Csr Ac;
    {
      const Csr AP = spgemm(A, P);
      Ac = spgemm(R, AP);
    }
    const bool cut = part && c->amg.empty();  // the level-0 transfer of a partition
    Csr Pl, Rl;
    if (cut) {  // the owned fine rows of P_0
      Pl.n = nrow;
      Pl.m = P.m;
      Pl.ptr.assign((size_t)nrow + 1, 0);
      for (int64_t i = 0; i < nrow; ++i) Pl.ptr[i + 1] = Pl.ptr[i] + (P.ptr[row0 + i + 1] - P.ptr[row0 + i]);
      Pl.col.assign(P.col.begin() + P.ptr[row0], P.col.begin() + P.ptr[row0 + nrow]);
      Pl.val.assign(P.val.begin() + P.ptr[row0], P.val.begin() + P.ptr[row0 + nrow]);
      Rl = transpose(Pl);
    }
    c->amg.emplace_back();
    AmgLevel& L = c->amg.back();
    L.n = na;
    // P and R: SELL-64 with float32 values; R's rows (one per aggregate, their
    // lengths vary with the aggregate) sorted by length inside windows of
    // kAmgSortWindow rows, P's kept in order (its outputs are the fine vectors:
    // a sorted P would scatter three fine streams).  One row per lane in CSR
    // left the wave's loads uncoalesced (measured slower, 475 vs 411 us per V-cycle)
    if (int e = upload_mat(c, cut ? Pl : P, L.P, false, true, 0, &L.p_nnz)) return e;
    if (int e = upload_mat(c, cut ? Rl : R, L.R, false, true, kAmgSortWindow, &L.r_nnz)) return e;
    if (int e = upload_mat(c, Ac, L.A, false, false, 0, &L.a_nnz)) return e;
    // a geometric level's operator is a 27-point stencil of a structured grid:
    // applied as a half stencil (112 B per row instead of ~12 B x 27 of SELL)
    if (grid) half_stencil(c, Ac, dims, L.sg);
    // level 0's transfers by index arithmetic (stored as SELL they were the
    // cycle's largest streams: V-cycle 472-475 -> 320-324 us at distorted C4)
    if (grid && c->amg.size() == 1 && !part) {
      L.geo0 = true;
      for (int a = 0; a < 3; ++a) {
        L.gfine[a] = fdims[a];
        L.gcoarse[a] = dims[a];
      }
    }
    const std::vector<double> dc = diag_inv(Ac);
    for (double v : dc)
      if (!(v > 0.0) || !std::isfinite(v)) return c->fail(TV_ERR_ARG, "AMG: coarse operator not positive definite");
    L.omega = 2.0 / (1.1 * lam_max(Ac, dc, 20));
    if (int e = amg_upload(c, dc, &L.dinv)) return e;
    for (double** v : {&L.b, &L.x, &L.w})
      if (int e = amg_alloc(c, (size_t)na, v)) return e;
    A = std::move(Ac);
  }
  if (c->amg.empty()) return c->fail(TV_ERR_ARG, "AMG: the mesh is too small to coarsen");
  HIPC(hipMalloc(&c->mgx, sizeof(double) * (size_t)std::max<int64_t>(1, c->nT)));
  HIPC(hipMemset(c->mgx, 0, sizeof(double) * (size_t)std::max<int64_t>(1, c->nT)));
  c->amg_on = true;
  c->mg_on = true;
  c->mg_omega0 = 0.0;  // the level-0 weight: lazily, at the temperature of the first solve (mg_dg_weight)
  return TV_OK;
}

int amg_setup(Ctx* c) {
  if (!c->um || c->n_parts > 1) return c->fail(TV_ERR_ARG, "AMG: unstructured meshes on one partition");
  Csr A;
  if (int e = fine_csr(c, A)) return e;
  const int64_t n = A.n;
  if (c->umg.J14 != nullptr) {  // structured topology (tv_um.hip): geometric transfers
    const int64_t grid[3] = {c->umg.s1, c->umg.s2 / c->umg.s1, c->umg.nv / c->umg.s2};
    return amg_build(c, std::move(A), 0, n, grid);
  }
  return amg_build(c, std::move(A), 0, n);
}

// The hierarchy of a partition of a distributed unstructured mesh (collective,
// at its first solve, once the communicator is set).  Every rank gathers the
// GLOBAL fine operator in the partition-major numbering -- its owned rows with
// global column ids (the ghosts' ids from their owners through the halo),
// summed into zero-filled global arrays by vector all-reduces (each row comes
// from one rank: the sums are exact) -- and builds the same hierarchy from it
// (the host setup is deterministic), PCGAMG's agglomeration of the coarse
// levels onto every process in the extreme: the V-cycle below level 0 runs
// replicated, one all-reduce of the level-1 right-hand side per application.
int amg_setup_part(Ctx* c) {
  if (!c->um || c->n_parts < 2) return c->fail(TV_ERR_ARG, "AMG: partitioned unstructured meshes");
  Csr Al;
  if (int e = fine_csr(c, Al)) return e;  // owned rows, local columns
  const int64_t nown = c->ownT_n, nloc = c->nT, off = c->globT_off;
  hipStream_t s = c->stream;
  double* dv = nullptr;
  auto dev = [&](size_t n) -> int {
    if (dv) HIPC(hipFree(dv));
    dv = nullptr;
    HIPC(hipMalloc(&dv, sizeof(double) * std::max<size_t>(1, n)));
    return TV_OK;
  };
  auto run = [&]() -> int {
    // global ids of the local vertices
    std::vector<double> gid((size_t)nloc, -1.0);
    for (int64_t i = 0; i < nown; ++i) gid[(size_t)i] = (double)(off + i);
    if (int e = dev((size_t)nloc)) return e;
    HIPC(hipMemcpyAsync(dv, gid.data(), sizeof(double) * (size_t)nloc, hipMemcpyHostToDevice, s));
    if (int e = halo_um(c, dv)) return e;
    HIPC(hipMemcpyAsync(gid.data(), dv, sizeof(double) * (size_t)nloc, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    for (double g : gid)
      if (!(g >= 0.0)) return c->fail(TV_ERR_STATE, "AMG: a ghost vertex received no global id");
    // global row count and row lengths
    double nn = (double)nown;
    if (int e = dev(1)) return e;
    HIPC(hipMemcpyAsync(dv, &nn, sizeof(double), hipMemcpyHostToDevice, s));
    if (int e = allreduce_vec(c, dv, 1)) return e;
    HIPC(hipMemcpyAsync(&nn, dv, sizeof(double), hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    const int64_t N = (int64_t)nn;
    // every rank holds the global CSR on the host (~27 entries x 16 B per row,
    // plus the hierarchy): 20M rows ~ 9 GB per rank before setup temporaries
    constexpr int64_t kAmgPartMaxRows = 20000000;
    if (N > kAmgPartMaxRows)
      return c->fail(TV_ERR_ARG, "AMG on a partitioned mesh gathers the global operator on every rank: at most 20M "
                                 "global vertices (use Jacobi beyond)");
    std::vector<double> len((size_t)N, 0.0);
    for (int64_t i = 0; i < nown; ++i) len[(size_t)(off + i)] = (double)(Al.ptr[i + 1] - Al.ptr[i]);
    if (int e = dev((size_t)N)) return e;
    HIPC(hipMemcpyAsync(dv, len.data(), sizeof(double) * (size_t)N, hipMemcpyHostToDevice, s));
    if (int e = allreduce_vec(c, dv, N)) return e;
    HIPC(hipMemcpyAsync(len.data(), dv, sizeof(double) * (size_t)N, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    Csr A;
    A.n = A.m = N;
    A.ptr.assign((size_t)N + 1, 0);
    for (int64_t r = 0; r < N; ++r) A.ptr[r + 1] = A.ptr[r] + (int64_t)len[(size_t)r];
    const int64_t nnz = A.ptr[N];
    // columns (global ids, ascending per row) and values of the owned rows
    std::vector<double> cv((size_t)nnz, 0.0), vv((size_t)nnz, 0.0);
    std::vector<std::pair<int64_t, double>> row;
    for (int64_t i = 0; i < nown; ++i) {
      row.clear();
      for (int64_t k = Al.ptr[i]; k < Al.ptr[i + 1]; ++k) row.emplace_back((int64_t)gid[(size_t)Al.col[k]], Al.val[k]);
      std::sort(row.begin(), row.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
      const int64_t o = A.ptr[off + i];
      for (size_t q = 0; q < row.size(); ++q) {
        cv[(size_t)o + q] = (double)row[q].first;
        vv[(size_t)o + q] = row[q].second;
      }
    }
    if (int e = dev((size_t)nnz)) return e;
    for (std::vector<double>* v : {&cv, &vv}) {
      HIPC(hipMemcpyAsync(dv, v->data(), sizeof(double) * (size_t)nnz, hipMemcpyHostToDevice, s));
      if (int e = allreduce_vec(c, dv, nnz)) return e;
      HIPC(hipMemcpyAsync(v->data(), dv, sizeof(double) * (size_t)nnz, hipMemcpyDeviceToHost, s));
      HIPC(hipStreamSynchronize(s));
    }
    A.col.resize((size_t)nnz);
    A.val.swap(vv);
    for (int64_t k = 0; k < nnz; ++k) A.col[(size_t)k] = (int)cv[(size_t)k];
    if (dv) HIPC(hipFree(dv));
    dv = nullptr;
    return amg_build(c, std::move(A), off, nown);
  };
  const int e = run();
  if (dv) hipFree(dv);
  return e;
}

// the V-cycle on coarse level l >= 1 (c->amg[l - 1]); its pre-smoothing step
// from 0 was formed by the restriction into it.  Returns the level's result.
static const double* amg_level(Ctx* c, size_t l) {
  AmgLevel& L = c->amg[l - 1];
  if (l == c->amg.size()) return L.x;  // coarsest: one Jacobi step
  AmgLevel& C = c->amg[l];
  hipStream_t s = c->stream;
  const bool sg = L.sg.J14 != nullptr;
  if (sg) launch_sg_apply(L.sg, c->st, L.x, nullptr, nullptr, 0.0, L.w, s);
  else launch_amg_apply(L.A, c->st, L.x, L.w, s);
  launch_amg_restrict(C.R, c->st, L.b, L.w, C.dinv, C.omega, C.b, C.x, s);
  const double* xc = amg_level(c, l + 1);
  launch_amg_prolong(C.P, c->st, xc, L.x, L.x, s);
  if (sg) launch_sg_apply(L.sg, c->st, L.x, L.b, L.dinv, L.omega, L.w, s);
  else launch_amg_post(L.A, c->st, L.x, L.b, L.dinv, L.omega, L.w, s);
  return L.w;
}

// z = omega0 D^-1 r (x0 = c->mgx, formed by k_mg_update) + P_0 V_1(P_0^T r),
// with the (z.z, z.r) records and the KSPCG tail
int amg_apply0(Ctx* c, const RedTail* tail) {
  AmgLevel& L1 = c->amg[0];
  if (c->n_parts > 1) {  // the partial restriction of the owned fine rows, summed over the ranks
    launch_amg_restrict(L1.R, c->st, c->r, nullptr, nullptr, 0.0, L1.b, nullptr, c->stream);
    if (int e = allreduce_vec(c, L1.b, L1.n)) return -e;
    launch_mg_jacobi(L1.n, c->st, L1.b, nullptr, nullptr, L1.dinv, L1.omega, L1.x, 0, c->stream);
  } else if (L1.geo0) {
    launch_geo_restrict0(L1.gfine, L1.gcoarse, c->st, c->r, L1.dinv, L1.omega, L1.b, L1.x, c->stream);
  } else {
    launch_amg_restrict(L1.R, c->st, c->r, nullptr, L1.dinv, L1.omega, L1.b, L1.x, c->stream);
  }
  const double* x1 = amg_level(c, 1);
  if (L1.geo0)
    return launch_geo_prolong0(L1.gfine, L1.gcoarse, c->st, x1, c->mgx, c->r, c->z, c->partials, tail, c->stream);
  return launch_amg_prolong0(L1.P, c->st, x1, c->mgx, c->r, c->z, c->partials, tail, c->stream);
}

// algorithmic bytes of one V-cycle (tv_kernel_bytes 11): the stored entries
// of every launched operator (A: 12 B, value + column; P, R: 8 B, float value
// + column; SELL padding included) and the
// vectors each launch streams once (gathered vectors counted once)
double amg_cycle_bytes(const Ctx* c) {
  const double n0 = (double)c->nT;
  const AmgLevel& L1 = c->amg[0];
  // R_0 (r in; b, x, dinv of level 1) and P_0 (x_1 in; x0, r in, z out): stored
  // transfers, or (geo0) applied by index arithmetic -- the vectors only
  const double t0 = L1.geo0 ? 0.0 : 8.0;
  double b = t0 * (double)L1.r_nnz + 8.0 * n0 + 24.0 * (double)L1.n;
  b += t0 * (double)L1.p_nnz + 8.0 * (double)L1.n + 24.0 * n0;
  for (size_t l = 0; l + 1 < c->amg.size(); ++l) {
    const AmgLevel& L = c->amg[l];
    const AmgLevel& C = c->amg[l + 1];
    const double n = (double)L.n, nc = (double)C.n;
    const double ab = L.sg.J14 ? 112.0 * n : 12.0 * (double)L.a_nnz;  // the operator: half stencil or SELL
    b += ab + 16.0 * n;                                          // w = A x
    b += 8.0 * (double)C.r_nnz + 16.0 * n + 24.0 * nc;           // b_c = R (b - w), x_c
    b += 8.0 * (double)C.p_nnz + 8.0 * nc + 16.0 * n;            // x += P x_c
    b += ab + 32.0 * n;                                          // post: x, b, dinv in, w out
  }
  return b;
}

}  // namespace tv
