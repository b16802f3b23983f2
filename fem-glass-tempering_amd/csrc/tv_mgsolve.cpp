// Geometric multigrid on the box hierarchy: setup, per-Newton preparation and
// the multigrid-preconditioned KSPCG (the reference's PCGAMG,
// ThermoViscoProblem.py:343-346, replaced for rectilinear 3D meshes).
#include <cstdlib>

#include "tv_ctx.h"

namespace tv {
constexpr int64_t kMgFoldFacesNodes = 4000000;  // level 0: facet terms folded into the restriction below this

// ---- geometric-multigrid preconditioned CG (options.preconditioner = GMG) ----
// Gershgorin bound of D^-1 J on a rectilinear level: max over nodes of the
// exact absolute row sum of the 27-point cell operator M + dt alpha K over its
// diagonal (the tensor-product entries from the per-axis 1D rows), over the
// distinct (row_x, row_y, row_z) combinations only.  The Robin facet rows are
// facet masses (row sum / diagonal <= 2.25 for Q1 facets): floor 2.25, then 5 %.
double mg_gershgorin(const std::vector<double> (&X)[3], double dt_alpha) {
  using Row = std::array<double, 6>;  // M lo / di / up, K lo / di / up
  std::vector<Row> rows[3];
  for (int s = 0; s < 3; ++s) {
    std::vector<double> cf;
    axis_coefs(X[s], 0, (int)X[s].size(), cf);
    for (size_t i = 0; i < X[s].size(); ++i) {
      const double* c = &cf[i * C_NCOEF];
      rows[s].push_back({c[C_MLO], c[C_MDI], c[C_MUP], c[C_KLO], c[C_KDI], c[C_KUP]});
    }
    std::sort(rows[s].begin(), rows[s].end());
    rows[s].erase(std::unique(rows[s].begin(), rows[s].end()), rows[s].end());
  }
  double b = 0.0;
  for (const Row& r0 : rows[0])
    for (const Row& r1 : rows[1])
      for (const Row& r2 : rows[2]) {
        double sum = 0.0, diag = 0.0;
        for (int a = 0; a < 3; ++a)
          for (int bb = 0; bb < 3; ++bb)
            for (int cc = 0; cc < 3; ++cc) {
              const double v = r0[a] * r1[bb] * r2[cc] +
                               dt_alpha * (r0[3 + a] * r1[bb] * r2[cc] + r0[a] * r1[3 + bb] * r2[cc] +
                                           r0[a] * r1[bb] * r2[3 + cc]);
              sum += std::fabs(v);
              if (a == 1 && bb == 1 && cc == 1) diag = v;
            }
        b = std::max(b, sum / diag);
      }
  return std::max(b, 2.25) * 1.05;
}

double mg_omega(double b) { return 2.0 / (1.1 * b); }

// the hierarchy below the fine grid (single partition, 3D CG1 marching path)
// the CG1 level of the box given by X (single partition), its vectors and weight
int mg_add_cg_level(Ctx* c, const std::vector<double> (&X)[3], double da) {
  c->mg.emplace_back();
  MgLevel& L = c->mg.back();
  for (int s = 0; s < 3; ++s) L.X[s] = X[s];
  if (int e = build_cg_grid(c, 3, L.X, 0, (int)L.X[2].size(), 0, 0, true, true, L.g, L.coef, &L.bnodes, L.ffbuf))
    return e;
  if (int e = mg_level_vectors(c, L)) return e;
  L.omega = mg_omega(mg_gershgorin(L.X, da));
  return TV_OK;
}

// lambda_max(B^-1 J) of the DG1 operator by power iteration, B the cell blocks;
// SIPG rows have no closed-form
// Gershgorin bound here.  The smoother takes it with a 21 % margin
int mg_dg_lambda(Ctx* c, const double* T, double* lam) {
  // a partition of a distributed unstructured mesh (collective): its owned rows,
  // the start vector's entries at their partition-major global indices, the
  // ghosts refreshed before every product, the norms all-reduced
  const bool part = c->n_parts > 1;
  const int64_t n = part ? c->ownT_n : c->nT;
  std::vector<double> h((size_t)n);
  uint64_t st = 0x9E3779B97F4A7C15ull;
  double nrm = 0.0;
  const int64_t skip = part ? c->globT_off : 0;
  for (int64_t t = 0; t < skip + n; ++t) {  // fixed-seed xorshift start vector in (0.5, 1.5)
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    if (t < skip) continue;
    h[(size_t)(t - skip)] = 0.5 + (double)(st >> 11) * (1.0 / 9007199254740992.0);
    nrm += h[(size_t)(t - skip)] * h[(size_t)(t - skip)];
  }
  auto gsum = [&](double& v) -> int {  // sum over the ranks (partitioned)
    if (!part) return TV_OK;
    HIPC(hipMemcpyAsync(c->sums + 4, &v, sizeof(double), hipMemcpyHostToDevice, c->stream));
    if (int e = allreduce(c, c->sums + 4, 1)) return e;
    HIPC(hipMemcpyAsync(&v, c->sums + 4, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    return TV_OK;
  };
  if (int e = gsum(nrm)) return e;
  for (double& v : h) v /= std::sqrt(nrm);
  HIPC(hipMemcpyAsync(c->mgx, h.data(), sizeof(double) * (size_t)n, hipMemcpyHostToDevice, c->stream));
  if (c->dggface) launch_dg_gface(c->dg, T, c->dggface, c->stream);
  else if (!c->um) launch_dg_diag(c->dg, T, c->dinv, 1, c->stream);
  std::vector<double> prt(1024);
  double l = 0.0;
  if (c->um) op_diag(c, T, c->dinv, 1);  // the algebraic multigrid's level 0: point Jacobi of J(T)
  for (int it = 0; it < 30; ++it) {
    if (part)
      if (int e = halo(c, c->mgx)) return e;
    op_japply(c, T, c->mgx, c->w, nullptr, nullptr);
    if (c->dggface) launch_dg_bsmooth(c->dg, nullptr, c->w, nullptr, c->dggface, 1.0, c->w, 0, c->stream);  // in place, per cell
    const int nb = launch_mg_pow(n, c->dggface ? nullptr : c->dinv, c->w, c->partials, c->stream);
    HIPC(hipMemcpyAsync(prt.data(), c->partials, sizeof(double) * (size_t)nb, hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    double s2 = 0.0;
    for (int b = 0; b < nb; ++b) s2 += prt[(size_t)b];
    if (int e = gsum(s2)) return e;
    l = std::sqrt(s2);  // ||D^-1 J x|| with ||x|| = 1
    if (!(l > 0.0) || !std::isfinite(l)) return c->fail(TV_ERR_HIP, "GMG: DG eigenvalue estimate failed");
    launch_mg_scale(n, c->w, 1.0 / l, c->mgx, c->stream);
  }
  *lam = l;
  return TV_OK;
}

// The DG level-0 smoother weight omega0 = 2 / (1.21 lambda_max) is estimated
// lazily, at the first multigrid solve (or V-cycle application), from the
// temperature it will precondition -- the Robin term 4 a_rad T^3 of the cell
// blocks vanishes at the T = 0 a freshly created context holds
int mg_dg_weight(Ctx* c, const double* T) {
  if (!(c->mg_dg || c->amg_on) || c->mg_omega0 > 0.0) return TV_OK;
  double lam = 0.0;
  if (int e = mg_dg_lambda(c, T, &lam)) return e;
  // AMG level 0 (additive point Jacobi): the coarse levels' 2 / (1.1 lambda)
  c->mg_omega0 = c->amg_on ? 2.0 / (1.1 * lam) : 2.0 / (1.1 * 1.1 * lam);
  return TV_OK;
}

// Coarsening rule of the box hierarchy (identical for a whole box and for its
// partitions, which plan it over the global grid): every other node kept
// along each axis with at least two cells, plus the last node when the cell
// count is odd (coarse nodes are a subset of the fine ones); stop where the
// operator is mass-dominated (dt alpha / h^2 <= 0.5 with h the smallest mean
// cell length: a Jacobi step is then a good solve) or nothing coarsens.
bool mg_next_level(const std::vector<double> (&Xp)[3], double da, bool automatic, std::vector<double> (&Xc)[3],
                   std::vector<char> (&is_c)[3], int coarse[3]) {
  double h = 1e300;
  bool any = false;
  for (int s = 0; s < 3; ++s) {
    const int cells = (int)Xp[s].size() - 1;
    coarse[s] = cells >= 2;
    any = any || coarse[s];
    if (cells >= 1) h = std::min(h, (Xp[s].back() - Xp[s].front()) / cells);
  }
  if (!any || (automatic && da / (h * h) <= 0.5)) return false;
  for (int s = 0; s < 3; ++s) {
    const int nf = (int)Xp[s].size();
    Xc[s].clear();
    is_c[s].assign(nf, 1);
    if (!coarse[s]) {
      Xc[s] = Xp[s];
      continue;
    }
    for (int i = 0; i < nf; ++i) is_c[s][i] = (i % 2 == 0 || i == nf - 1) ? 1 : 0;
    for (int i = 0; i < nf; ++i)
      if (is_c[s][i]) Xc[s].push_back(Xp[s][i]);
  }
  return true;
}

// Transfer tables of one axis over the whole (global) axis: prolongation = two
// (coarse index, weight) pairs per fine node (exact linear interpolation),
// restriction R = P^T = three (fine index, weight) pairs per coarse node
void mg_axis_tables(const std::vector<double>& Xf, const std::vector<char>& is_c, std::vector<int>& pi,
                    std::vector<double>& pw, std::vector<int>& ri, std::vector<double>& rw) {
  const int nf = (int)Xf.size();
  std::vector<int> cpos(nf, -1), fpos;
  for (int i = 0; i < nf; ++i)
    if (is_c[i]) {
      cpos[i] = (int)fpos.size();
      fpos.push_back(i);
    }
  const int nc = (int)fpos.size();
  pi.assign(2 * (size_t)nf, 0);
  pw.assign(2 * (size_t)nf, 0.0);
  ri.assign(3 * (size_t)nc, 0);
  rw.assign(3 * (size_t)nc, 0.0);
  for (int i = 0; i < nf; ++i) {
    if (is_c[i]) {
      pi[2 * i] = pi[2 * i + 1] = cpos[i];
      pw[2 * i] = 1.0;
    } else {  // linear interpolation between the coarse neighbours i - 1 and i + 1
      const double wl = (Xf[i + 1] - Xf[i]) / (Xf[i + 1] - Xf[i - 1]);
      pi[2 * i] = cpos[i - 1];
      pi[2 * i + 1] = cpos[i + 1];
      pw[2 * i] = wl;
      pw[2 * i + 1] = 1.0 - wl;
    }
  }
  for (int I = 0; I < nc; ++I) {  // R = P^T: the fine nodes that interpolate from I
    const int fc = fpos[I];
    for (int q = 0; q < 3; ++q) ri[3 * I + q] = fc;
    rw[3 * I + 1] = 1.0;
    if (fc - 1 >= 0 && !is_c[fc - 1]) {
      ri[3 * I] = fc - 1;
      rw[3 * I] = pw[2 * (fc - 1) + 1];  // fine fc - 1: its right coarse neighbour is I
    }
    if (fc + 1 < nf && !is_c[fc + 1]) {
      ri[3 * I + 2] = fc + 1;
      rw[3 * I + 2] = pw[2 * (fc + 1)];  // fine fc + 1: its left coarse neighbour is I
    }
  }
}

// Tables of the fused residual restriction (RRArgs) along one axis: for coarse
// node I (fine node fc = ri[3I + 1]) the window fc - 2 .. fc + 2 and the weights
// of (R M), (R K) and R over it, from the fine 1D rows and the restriction
// weights.  False when a product reaches outside the window (not a nested pair).
static bool rr_axis(const std::vector<double>& Xf, const std::vector<int>& ri, const std::vector<double>& rw,
                    std::vector<int>& f0, std::vector<double>& w) {
  const int nf = (int)Xf.size(), nc = (int)ri.size() / 3;
  std::vector<double> cf;
  axis_coefs(Xf, 0, nf, cf);
  f0.assign(nc, 0);
  w.assign(15 * (size_t)nc, 0.0);
  for (int I = 0; I < nc; ++I) {
    f0[I] = ri[3 * I + 1] - 2;
    for (int q = 0; q < 3; ++q) {
      const int f = ri[3 * I + q];
      const double wt = rw[3 * I + q];
      if (wt == 0.0) continue;
      const double* cc = &cf[(size_t)f * C_NCOEF];
      auto add = [&](int col, int fi, double v) -> bool {
        if (v == 0.0) return true;
        const int m = fi - f0[I];
        if (fi < 0 || fi >= nf || m < 0 || m > 4) return false;
        w[15 * (size_t)I + 5 * col + m] += wt * v;
        return true;
      };
      if (!(add(0, f - 1, cc[C_MLO]) && add(0, f, cc[C_MDI]) && add(0, f + 1, cc[C_MUP]) &&
            add(1, f - 1, cc[C_KLO]) && add(1, f, cc[C_KDI]) && add(1, f + 1, cc[C_KUP]) && add(2, f, 1.0)))
        return false;
    }
  }
  return true;
}

// The fused residual restriction from fine coordinates Xp into coarse level L
// (single partition): x needs even fine cell counts (lanes own fine pairs
// 2I, 2I + 1), the march axis consecutive windows two fine planes apart (every
// coarsened axis: the odd tail's window too); the row axis is free.
static int rr_setup(Ctx* c, MgLevel& L, const std::vector<double> (&Xp)[3], const std::vector<int> (&ri)[3],
                    const std::vector<double> (&rw)[3]) {
  RRArgs& a = L.rr;
  a = RRArgs{};
  const MgXfer& x = L.xf;
  if (!x.coarse[0] || x.fn[0] < 5 || !(x.fn[0] & 1)) return TV_OK;
  std::vector<int> f0[3];
  std::vector<double> w[3];
  for (int s = 0; s < 3; ++s)
    if (!rr_axis(Xp[s], ri[s], rw[s], f0[s], w[s])) return TV_OK;
  auto regular = [&](int s) {
    if (!x.coarse[s] || x.cn[s] < 2) return false;
    for (int I = 0; I + 1 < x.cn[s]; ++I)
      if (f0[s][I + 1] - f0[s][I] != 2) return false;
    return true;
  };
  int qa = (x.cn[1] <= x.cn[2]) ? 1 : 2;
  if (!regular(qa)) qa = 3 - qa;
  if (!regular(qa)) return TV_OK;
  a.raxis = 3 - qa;
  for (int I = 0; I + 1 < x.cn[a.raxis]; ++I)  // the row axis: windows 1 or 2 fine rows apart (slab bound)
    if (f0[a.raxis][I + 1] - f0[a.raxis][I] > 2) return TV_OK;
  for (int s = 0; s < 3; ++s) {
    a.fn[s] = x.fn[s];
    a.cn[s] = x.cn[s];
    if (int e = mg_upload(c, L, f0[s], &a.ax[s].f0)) return e;
    if (int e = mg_upload(c, L, w[s], &a.ax[s].w)) return e;
  }
  a.da = L.g.dt_alpha;
  a.nseg = (x.cn[0] + 61) / 62;
  // chunks of the march axis: about `target` workgroups of 8 waves (2 fit a CU:
  // 67 KB of LDS each), >= 3 coarse planes per chunk (TVFEM_RR_WG overrides)
  // (256 measured best at C4: V-cycle 226 us against 240 / 231 us at 128 / 512)
  const char* te = std::getenv("TVFEM_RR_WG");
  const int target = te ? std::max(1, std::atoi(te)) : 256;
  const int64_t rowblocks = (x.cn[a.raxis] + 7) / 8;
  a.qchunk = std::min(x.cn[qa], 64);  // <= kRRQMax (tv_mg.hip)
  while ((int64_t)a.nseg * rowblocks * ((x.cn[qa] + a.qchunk - 1) / a.qchunk) < target && a.qchunk > 3)
    a.qchunk = (a.qchunk + 1) / 2;
  a.on = 1;
  return TV_OK;
}

// Levels whose restriction runs fused (bit l: from level l into level l + 1):
// level 0 on fine grids of >= kRRMinNodes nodes.  Measured (C4, 8.2M nodes,
// interleaved): V-cycle 249 -> 226 us, step 10.22 -> 9.85 ms; at C3 (1M nodes)
// 3.15 -> 3.21 ms and on the coarse levels slower (their J x launches are
// latency-bound, the facet launch adds one), so not there.  TVFEM_MG_RR (a bit
// mask, read at setup) overrides, for tests and A/B measurement.
constexpr int64_t kRRMinNodes = 3000000;
static unsigned rr_levels(int64_t fine_nodes) {
  const char* e = std::getenv("TVFEM_MG_RR");
  if (e) return (unsigned)std::strtoul(e, nullptr, 0);
  return fine_nodes >= kRRMinNodes ? 1u : 0u;
}

// T, b, x, w, dinv of a level (local size L.n), zeroed
int mg_level_vectors(Ctx* c, MgLevel& L) {
  const CgGrid& f = c->cg;  // thermal constants (set by setup_mesh for both families)
  L.g.dt = f.dt; L.g.dt_alpha = f.dt_alpha; L.g.dt_f = f.dt_f;
  L.g.a_rad = f.a_rad; L.g.a_conv = f.a_conv; L.g.T_amb = f.T_amb; L.g.T_amb4 = f.T_amb4;
  L.n = (int64_t)L.g.n0 * L.g.n1 * L.g.n2;
  for (double** q : {&L.T, &L.b, &L.x, &L.w, &L.dinv}) {
    void* p = nullptr;
    HIPC(hipMalloc(&p, sizeof(double) * (size_t)std::max<int64_t>(1, L.n)));
    HIPC(hipMemsetAsync(p, 0, sizeof(double) * (size_t)std::max<int64_t>(1, L.n), c->stream));
    L.bufs.push_back(p);
    *q = static_cast<double*>(p);
  }
  return TV_OK;
}

int mg_setup(Ctx* c) {
  const bool dg = c->fam_T == TV_DG;
  if (c->dim != 3 || c->um || (!dg && !cg_cgs_supported(c->cg)) || (dg && (c->dg.deg1 || c->dg.deg2)))
    return c->fail(TV_ERR_ARG, "preconditioner GMG: 3D CG1 or DG1 temperature space on a rectilinear mesh only");
  if (c->cgs) return c->fail(TV_ERR_ARG, "preconditioner GMG runs in the KSPCG form (pcg_variant KSPCG or AUTO)");
  if (c->n_parts > 1 && !dg) return mg_setup_dist(c);  // slab-partitioned CG1 box (tv_mgdist.cpp)
  // a DG1 box, one partition or slab-partitioned: level 1 is the CG1 space of
  // the WHOLE box (the global coordinates), and it and every coarser level are
  // replicated on every slab (mg_A = 1): a slab restricts its owned cells into
  // the vertex planes they touch, one all-reduce of the level-1 vector sums the
  // shared planes, every slab runs the CG cycle below and prolongs into all its
  // local cells (ghost layers included: the level holds every vertex)
  if (c->n_parts > 1) c->mg_A = 1;
  std::vector<double> tmp, Xf[3];
  for (int s = 0; s < 3; ++s) Xf[s] = storage_coords(c, s, tmp);
  const double da = c->P.dt * c->P.alpha;
  HIPC(hipMalloc(&c->mgx, sizeof(double) * (size_t)std::max<int64_t>(1, c->nT)));
  HIPC(hipMemsetAsync(c->mgx, 0, sizeof(double) * (size_t)std::max<int64_t>(1, c->nT), c->stream));
  if (dg) {
    // level 1: the CG1 space of the same box (two-level DG -> CG, then the CG hierarchy)
    c->mg_dg = true;
    HIPC(hipMalloc(&c->dggface, sizeof(double) * (size_t)dg_gface_size(c->dg)));
    c->mg_omega0 = 0.0;  // estimated at the first solve, at its T (mg_dg_weight)
    if (int e = mg_add_cg_level(c, Xf, da)) return e;
  } else {
    c->mg_omega0 = mg_omega(mg_gershgorin(Xf, da));
  }
  const int max_levels = c->O.mg_levels > 0 ? c->O.mg_levels : 8;
  const bool automatic = c->O.mg_levels <= 0;
  std::vector<double> Xp[3] = {Xf[0], Xf[1], Xf[2]};
  for (int lev = 1 + (dg ? 1 : 0); lev < max_levels; ++lev) {
    std::vector<double> Xc[3];
    std::vector<char> is_c[3];  // fine node kept on this level
    int coarse[3];
    if (!mg_next_level(Xp, da, automatic, Xc, is_c, coarse)) break;
    c->mg.emplace_back();
    MgLevel& L = c->mg.back();
    for (int s = 0; s < 3; ++s) L.X[s] = Xc[s];
    if (int e = build_cg_grid(c, 3, L.X, 0, (int)L.X[2].size(), 0, 0, true, true, L.g, L.coef, &L.bnodes, L.ffbuf))
      return e;
    if (int e = mg_level_vectors(c, L)) return e;
    L.omega = mg_omega(mg_gershgorin(L.X, da));
    // transfer maps (finer level Xp -> this level)
    MgXfer& x = L.xf;
    std::vector<int> ri[3];
    std::vector<double> rw[3];
    for (int s = 0; s < 3; ++s) {
      std::vector<int> pi;
      std::vector<double> pw;
      mg_axis_tables(Xp[s], is_c[s], pi, pw, ri[s], rw[s]);
      if (int e = mg_upload(c, L, pi, &x.pi[s])) return e;
      if (int e = mg_upload(c, L, pw, &x.pw[s])) return e;
      if (int e = mg_upload(c, L, ri[s], &x.ri[s])) return e;
      if (int e = mg_upload(c, L, rw[s], &x.rw[s])) return e;
      x.fn[s] = (int)Xp[s].size();
      x.cn[s] = (int)L.X[s].size();
      x.coarse[s] = coarse[s];
    }
    x.f_kb = 0;
    x.f_ke = x.fn[2];
    x.c_kb = 0;
    x.c_ke = x.cn[2];
    x.aligned = 1;
    // the fused residual restriction into this level (CG levels of a CG box;
    // the DG1 -> CG1 transfer is the cell-vertex one)
    const size_t from = c->mg.size() - 1 - (dg ? 1 : 0);  // index of the finer level (0: the fine grid)
    if (!dg && ((rr_levels(c->nT) >> from) & 1u))
      if (int e = rr_setup(c, L, Xp, ri, rw)) return e;
    for (int s = 0; s < 3; ++s) Xp[s] = L.X[s];
  }
  c->mg_on = true;
  return TV_OK;
}

// per Newton iteration: T injected down the hierarchy (DG: the vertex mean of
// the cell-local values onto the CG level), coarse Jacobi diagonals

int mg_prepare(Ctx* c, const double* T) {
  if (c->amg_on) return TV_OK;  // the algebraic hierarchy is T-independent (tv_amg.cpp)
  // a DG1 slab: level 1's T = the vertex means on its owned vertex planes,
  // summed over the slabs into the replicated vector (each plane from one slab)
  const bool dgpart = c->mg_dg && c->n_parts > 1;
  auto dg_T = [&](MgLevel& L) -> int {
    if (!dgpart) {
      launch_mg_dg_T(c->dg, T, L.T, 0, c->stream);
      return TV_OK;
    }
    HIPC(hipMemsetAsync(L.T, 0, sizeof(double) * (size_t)L.n, c->stream));
    launch_mg_dg_T(c->dg, T, L.T, c->plane_begin - c->dg.k_begin, c->stream);
    return allreduce_vec(c, L.T, L.n);
  };
  // after the first call (dinv interiors in place): the CG levels below the
  // base in two launches (launch_mg_prepare)
  const size_t base = c->mg_dg ? 1 : 0;  // DG: level 1 is the vertex mean of the DG field
  const size_t ncg = c->mg.size() - std::min(c->mg.size(), base);
  bool ready = ncg > 0 && ncg <= (size_t)kMgPrepMax;
  for (size_t l = base; l < c->mg.size() && ready; ++l)
    ready = c->mg[l].dinv_interior && cg_uses_march(c->mg[l].g) && c->mg[l].g.bnodes != nullptr;
  if (ready) {
    if (base == 1) {
      MgLevel& L = c->mg[0];
      if (int e = dg_T(L)) return e;
      if (c->dggface) launch_dg_gface(c->dg, T, c->dggface, c->stream);
      launch_cg_diag(L.g, L.T, L.dinv, 1, c->stream, true);
    }
    MgPrep p{};
    p.nlev = (int)ncg;
    p.Tbase = base == 1 ? c->mg[0].T : T;
    for (size_t i = 0; i < ncg; ++i) {
      MgLevel& L = c->mg[base + i];
      p.xf[i] = L.xf;
      p.T[i] = L.T;
      p.dinv[i] = L.dinv;
      p.g[i] = L.g;
      p.off_n[i + 1] = p.off_n[i] + (L.n + 63) / 64 * 64;
      p.off_b[i + 1] = p.off_b[i] + (L.g.n_bnodes + 63) / 64 * 64;
    }
    launch_mg_prepare(p, c->stream);
    return TV_OK;
  }
  const double* Tf = T;
  for (size_t l = 0; l < c->mg.size(); ++l) {
    MgLevel& L = c->mg[l];
    if (l == 0 && c->mg_dg) {
      if (int e = dg_T(L)) return e;
      if (c->dggface) launch_dg_gface(c->dg, T, c->dggface, c->stream);
    }
    else launch_mg_inject(L.xf, Tf, L.T, c->stream);
    launch_cg_diag(L.g, L.T, L.dinv, 1, c->stream, L.dinv_interior);
    L.dinv_interior = true;
    Tf = L.T;
  }
  return TV_OK;
}

// V-cycle on coarse level l >= 1 (index l - 1 in c->mg): rhs b -> x; the
// pre-smoothing step from 0 (x = omega D^-1 b) was formed by the restriction
// that produced b.  The J x before the restriction is complete (k_cg_addfaces:
// a per-node facet term inside the 27-point gather measured slower); the one
// before the post-smoothing leaves the facet terms of the faces along the
// march to that pointwise consumer (FaceAdd).
// The prolongation from coarse level index ci (c->mg[ci]) into its finer level:
// where that level has a post-smoothing step (not the coarsest) and the
// 2 x 2 block prolongation runs, the step is applied on the fly (CoarsePost)
// and mg_level skipped its k_mg_jacobi launch.
void mg_prolong_from(Ctx* c, size_t ci, double* xf, const double* mask) {
  MgLevel& C = c->mg[ci];
  const bool smoothed = ci + 1 < c->mg.size() && mg_prolong_smooths(C.xf);
  if (smoothed) {
    const CoarsePost cp{C.b, C.w, C.dinv, C.omega, cg_face_add(C.g, 0)};
    launch_mg_prolong(C.xf, c->st, xf, C.x, mask, c->stream, &cp);
  } else {
    launch_mg_prolong(C.xf, c->st, xf, C.x, mask, c->stream);
  }
}

void mg_level(Ctx* c, size_t l) {
  MgLevel& L = c->mg[l - 1];
  hipStream_t s = c->stream;
  if (l < c->mg.size()) {
    const MgLevel& C = c->mg[l];
    const FaceAdd fa = cg_face_add(L.g, 0);
    if (C.rr.on && fa.on) {  // fused residual restriction (no J x of this level)
      launch_cg_facet_faces(L.g, L.T, L.x, c->st, s);
      launch_mg_rrestrict(C.rr, c->st, L.b, L.x, cg_face_add_all(L.g), C.b, C.dinv, C.omega, C.x, s);
    } else if (fa.on && mg_restrict_folds_faces(C.xf)) {  // the restriction adds the facet terms (no k_cg_addfaces)
      launch_cg_japply_partial(L.g, L.T, L.x, L.w, c->st, s);
      launch_mg_restrict(C.xf, c->st, L.b, L.w, &fa, nullptr, C.b, C.dinv, C.omega, C.x, s);
    } else {
      launch_cg_japply(L.g, L.T, L.x, L.w, nullptr, nullptr, s, c->st);
      launch_mg_restrict(C.xf, c->st, L.b, L.w, nullptr, nullptr, C.b, C.dinv, C.omega, C.x, s);
    }
    mg_level(c, l + 1);
    mg_prolong_from(c, l, L.x, nullptr);
    launch_cg_japply_partial(L.g, L.T, L.x, L.w, c->st, s);
    // post-smoothing, unless the prolongation out of this level applies it (mg_prolong_from)
    if (!mg_prolong_smooths(L.xf))
      launch_mg_jacobi(L.n, c->st, L.b, L.w, &fa, L.dinv, L.omega, L.x, 1, s);
  }
}

// level 0: x0 = omega dinv r is in c->mgx (k_mg_update); coarse correction,
// post-smoothing into z with the (z.z, z.r) reduction tail
int mg_apply0(Ctx* c, const double* T, const RedTail* tail) {
  if (c->amg_on) return amg_apply0(c, tail);
  const int64_t n = c->nT;
  hipStream_t s = c->stream;
  const double* mask = c->dir_on ? c->dinv : nullptr;  // Dirichlet: the free subspace
  if (c->mg_dg) {  // DG1 level 0: complete DG J x (Robin facets inline), vertex sums / injection to CG1
    const DgGrid& d = c->dg;
    MgLevel& C = c->mg[0];
    if (c->n_parts > 1) {  // a slab (mg_setup): the replicated level 1, see there
      const int kg0 = c->plane_begin - d.k_begin;
      if (int e = halo(c, c->mgx)) return -e;  // x0 of the ghost layers (J x0, the prolongation into them)
      launch_dg_japply(d, T, c->mgx, c->w, nullptr, nullptr, s, c->st);
      if (hipMemsetAsync(C.b, 0, sizeof(double) * (size_t)C.n, s) != hipSuccess)
        return -c->fail(TV_ERR_HIP, "GMG: level-1 memset");
      launch_mg_dg_restrict(d, c->st, c->r, c->w, mask, C.b, nullptr, 0.0, nullptr, kg0, s);
      if (int e = allreduce_vec(c, C.b, C.n)) return -e;
      launch_mg_jacobi(C.n, c->st, C.b, nullptr, nullptr, C.dinv, C.omega, C.x, 0, s);  // pre-smoothing from 0
      mg_level(c, 1);
      launch_mg_dg_prolong(d, c->st, c->mgx, C.x, mask, kg0, s);
    } else {
      launch_dg_japply(d, T, c->mgx, c->w, nullptr, nullptr, s, c->st);
      launch_mg_dg_restrict(d, c->st, c->r, c->w, mask, C.b, C.dinv, C.omega, C.x, 0, s);
      mg_level(c, 1);
      launch_mg_dg_prolong(d, c->st, c->mgx, C.x, mask, 0, s);
    }
    launch_dg_japply(d, T, c->mgx, c->w, nullptr, nullptr, s, c->st);
    if (c->dggface)
      return launch_dg_bpost(d, c->st, c->mgx, c->r, c->w, c->dggface, c->mg_omega0, c->z, c->partials, tail, s);
    return launch_mg_post(n, c->st, c->mgx, c->r, c->w, nullptr, c->dinv, c->mg_omega0, c->z, c->partials, tail, s);
  }
  const FaceAdd fa = cg_face_add(c->cg, 0);
  if (!c->mg.empty()) {
    MgLevel& C = c->mg[0];
    // below kMgFoldFacesNodes the restriction adds the face-workgroup facet
    // terms itself, as on the coarse levels (one launch fewer where the V-cycle
    // is launch-bound); at C4 a complete J x (k_cg_addfaces) measured the same
    if (C.rr.on && mask == nullptr && fa.on) {
      // b_1 = R (r - J x0) without J x0: the facet terms of x0 on every face,
      // then the fused residual restriction (RRArgs) with level 1's pre-smoothing
      launch_cg_facet_faces(c->cg, T, c->mgx, c->st, s);
      launch_mg_rrestrict(C.rr, c->st, c->r, c->mgx, cg_face_add_all(c->cg), C.b, C.dinv, C.omega, C.x, s);
    } else if (fa.on && mg_restrict_folds_faces(C.xf) && n < kMgFoldFacesNodes) {
      launch_cg_japply_partial(c->cg, T, c->mgx, c->w, c->st, s);
      launch_mg_restrict(C.xf, c->st, c->r, c->w, &fa, mask, C.b, C.dinv, C.omega, C.x, s);
    } else {
      launch_cg_japply(c->cg, T, c->mgx, c->w, nullptr, nullptr, s, c->st);
      launch_mg_restrict(C.xf, c->st, c->r, c->w, nullptr, mask, C.b, C.dinv, C.omega, C.x, s);
    }
    mg_level(c, 1);
    mg_prolong_from(c, 0, c->mgx, mask);
  }
  // J x, post-smoothing and (z.z, z.r) in the march epilogue (+ the side-face pass)
  {
    const int nrec = launch_cg_japply_post(c->cg, T, c->mgx, c->r, c->dinv, c->mg_omega0, c->z, c->st, c->partials,
                                           tail, s);
    if (nrec >= 0) return nrec;
  }
  launch_cg_japply_partial(c->cg, T, c->mgx, c->w, c->st, s);
  return launch_mg_post(n, c->st, c->mgx, c->r, c->w, &fa, c->dinv, c->mg_omega0, c->z, c->partials, tail, s);
}

int mg_iteration(Ctx* c, const double* T, int it) {
  const int64_t n = c->nT;
  const int slot = c->ts_next + it;
  uint64_t* ts = (c->ktime && (it % c->kstride) == 0 && slot < kTsCap) ? c->d_ts + 4 * slot : nullptr;
  RedTail t1{c->counters, c->partials, c->sums, c->st, 2, ts};
  int np = 0;
  if (!op_japply_fused(c, T, &np, &t1, it))  // p <- z + b p ; w <- J p ; p.w ; alpha
    if (int e = reduce_logic(c, np, 1, 2, 1)) return e;
  const FaceAdd fa = (c->mg_dg || c->um) ? FaceAdd{} : cg_face_add(c->cg, 0);  // DG, unstructured: w is complete
  if (c->dggface)
    launch_dg_bupdate(c->dg, c->st, c->pA, c->pB, c->w, c->dggface, c->mg_omega0, c->r, c->f[TV_F_DX].ptr, c->mgx, it, 0,
                      c->stream);
  else
    launch_mg_update(n, c->st, c->pA, c->pB, c->w, &fa, c->dinv, c->mg_omega0, c->r, c->f[TV_F_DX].ptr, c->mgx, it, 0,
                     c->stream);
  RedTail t2{c->counters + kTailCounters, c->partials, c->sums, c->st, 3, nullptr};
  mg_apply0(c, T, &t2);  // z <- V(r); z.z, z.r; beta, convergence
  return TV_OK;
}

int pcg_solve_mg(Ctx* c, const double* T, int* its, int* reason, bool post) {
  const int64_t n = c->nT;
  const PcgState h = pcg_state_init(c);
  // from pinned memory (an asynchronous upload; a pageable source is staged by
  // the runtime -- no step-time change measured at C2 / C3 / C4)
  c->h_st[2] = h;
  launch_set_state(c->st, h, c->stream, c->solve_gate);
  if (int e = mg_prepare(c, T)) return e;
  if (int e = mg_dg_weight(c, T)) return e;
  if (c->dggface)
    launch_dg_bupdate(c->dg, c->st, c->pA, c->pB, c->w, c->dggface, c->mg_omega0, c->r, c->f[TV_F_DX].ptr, c->mgx, 0, 1,
                      c->stream);  // dx <- 0, x0 <- omega B^-1 r
  else
    launch_mg_update(n, c->st, c->pA, c->pB, c->w, nullptr, c->dinv, c->mg_omega0, c->r, c->f[TV_F_DX].ptr, c->mgx, 0, 1,
                     c->stream);  // dx <- 0, x0 <- omega dinv r
  RedTail t0{c->counters + kTailCounters, c->partials, c->sums, c->st, 1, nullptr};
  mg_apply0(c, T, &t0);  // z <- V(r); dp, beta (KSPCG init)
  if (c->ktime && c->ts_next + c->O.ksp_max_it + 8 > kTsCap)
    if (int e = ts_flush(c)) return e;
  // an MG iteration is ~25 launches: the previous solve's count (hint) is queued
  // right behind the init, with no host wait in between (the GPU would idle
  // while the host enqueues ~100 launches; an init that already converged
  // makes every queued launch exit at once), then one iteration at a time
  // behind a poll.  The Newton solves of a step take near-constant counts, so
  // the hint usually ends the solve at the first poll.
  int launched = 0;
  auto enqueue = [&](int nb) -> int {
    for (int b = 0; b < nb; ++b)
      if (int e = mg_iteration(c, T, launched + b)) return e;
    launched += nb;
    HIPC(hipGetLastError());
    if (int e = publish(c, &c->h_st[0], c->st, sizeof(PcgState))) return e;
    HIPC(hipEventRecord(c->evp[0], c->stream));
    if (post) {  // the Newton iteration's next work, queued before the host's poll (it runs once)
      launch_post_group(n, c->st, c->pA, c->pB, c->f[TV_F_DX].ptr, c->f[TV_F_T].ptr, c->partials, c->sums, c->stream);
      if (int e = queue_newton_norm(c, c->sums)) return e;
    }
    return TV_OK;
  };
  const int hk = std::min(c->newton_k, 15);
  if (int e = enqueue(std::max(1, c->mg_hint[hk] > 0 ? c->mg_hint[hk] : c->pcg_hint))) return e;
  for (;;) {
    HIPC(hipEventSynchronize(c->evp[0]));
    if (c->h_st[0].done) break;
    if (launched > c->O.ksp_max_it + 2) return c->fail(TV_ERR_KSP, "PCG: iteration guard exceeded");
    if (int e = enqueue(1)) return e;
  }
  *its = c->h_st[0].it;
  *reason = c->h_st[0].reason;
  // level 0 updates dx in pairs of iterations from iteration 1 on (k_mg_update /
  // k_dg_bupdate DXU): solves of 0 / 1 iterations and the last step of an odd-length one
  if (!post) launch_mg_dx_finish(n, c->st, c->pA, c->pB, c->f[TV_F_DX].ptr, *its, c->stream);
  if (*reason != R_SKIPPED) {  // a solve gated off by the Newton test says nothing of the count
    c->pcg_hint = std::max(1, c->h_st[0].it);
    c->mg_hint[hk] = c->pcg_hint;
  }
  if (c->ktime) {
    for (int it = 0; it < *its; it += c->kstride)
      if (c->ts_next + it < kTsCap) c->ts_pending.push_back(c->ts_next + it);
    c->ts_next = std::min(kTsCap, c->ts_next + launched);
  }
  return TV_OK;
}

}  // namespace tv

using namespace tv;

// tv_precond_apply on a partition (collective: every rank calls it): the
// operator the partitioned Krylov solve applies, on this rank's owned dofs --
// Jacobi, or the partitioned V-cycle (GLOBAL: the distributed cycle of the
// whole box; LOCAL: this slab's own cycle)
static int precond_apply_part(Ctx* c, const double* r_dev, double* z_dev) {
  if (int e = require_comm(c, "tv_precond_apply")) return e;
  if (c->um || c->fam_T != TV_CG) return c->fail(TV_ERR_ARG, "tv_precond_apply: partitioned CG1 box meshes");
  const double* T = c->f[TV_F_T].ptr;
  const int64_t off = c->ownT_off, n = c->ownT_n;
  hipStream_t s = c->stream;
  if (int e = halo(c, c->f[TV_F_T].ptr)) return e;  // the PC setup reads the ghost planes' T (side-face facets)
  launch_cg_diag(c->cg, T, c->dinv, 1, s, c->dinv_interior);
  c->dinv_interior = true;
  if (c->dir_on) launch_bc_mask(c, c->dinv);
  if (!c->mg_on) {
    launch_mg_jacobi(n, nullptr, r_dev, nullptr, nullptr, c->dinv + off, 1.0, z_dev, 0, s);
  } else {
    PcgState h{};
    HIPC(hipMemcpyAsync(c->st, &h, sizeof(PcgState), hipMemcpyHostToDevice, s));
    if (int e = mg_prepare_dist(c, T)) return e;
    if (c->dir_on)
      if (int e = halo(c, c->dinv)) return e;
    if (c->mg_mask0) launch_mg_ownmask(c->nT, off, off + n, c->dir_on ? c->dinv : nullptr, c->mg_mask0, s);
    HIPC(hipMemcpyAsync(c->r + off, r_dev, sizeof(double) * (size_t)n, hipMemcpyDeviceToDevice, s));
    int64_t woff, nwin;  // deep ghosts: r on the ghost planes, x0 on the write window
    fine_window(c, &woff, &nwin);
    if (c->ghost_depth > 1)
      if (int e = halo(c, c->r)) return e;
    launch_mg_jacobi(nwin, c->st, c->r + woff, nullptr, nullptr, c->dinv + woff, c->mg_omega0, c->mgx + woff, 0, s);
    if (int e = mg_apply0_dist(c, T, nullptr)) return e;
    HIPC(hipMemcpyAsync(z_dev, c->z + off, sizeof(double) * (size_t)n, hipMemcpyDeviceToDevice, s));
  }
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(s));
  return TV_OK;
}

extern "C" {

int tv_precond_apply(void* ctx, const double* r_dev, double* z_dev) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !r_dev || !z_dev) return TV_ERR_ARG;
  hipSetDevice(c->device);
  HIPC(hipDeviceSynchronize());  // inputs written on other streams (header)
  if (c->n_parts > 1) return precond_apply_part(c, r_dev, z_dev);
  const double* T = c->f[TV_F_T].ptr;
  const int64_t n = c->nT;
  hipStream_t s = c->stream;
  // the PC setup of the Newton iteration at this T
  if (!c->dggface) {
    if (!c->um && c->fam_T == TV_CG) {
      launch_cg_diag(c->cg, T, c->dinv, 1, s, c->dinv_interior);
      c->dinv_interior = true;
    } else {
      op_diag(c, T, c->dinv, 1);
    }
  }
  // Dirichlet mode: the solve's preconditioner acts on the free subspace only
  // (dinv = 0 on the constrained rows, as k_bc_lift sets it before every solve;
  // the V-cycle masks its transfers with the same dinv)
  if (c->dir_on && c->fam_T == TV_CG) launch_bc_mask(c, c->dinv);
  if (c->mg_dg || c->amg_on)
    if (int e = mg_dg_weight(c, T)) return e;
  if (!c->mg_on) {
    launch_mg_jacobi(n, nullptr, r_dev, nullptr, nullptr, c->dinv, 1.0, z_dev, 0, s);  // z = dinv .* r
  } else {
    PcgState h{};  // running state: the V-cycle's kernels skip work once a solve is done
    HIPC(hipMemcpyAsync(c->st, &h, sizeof(PcgState), hipMemcpyHostToDevice, s));
    if (int e = mg_prepare(c, T)) return e;
    HIPC(hipMemcpyAsync(c->r, r_dev, sizeof(double) * (size_t)n, hipMemcpyDeviceToDevice, s));
    if (c->dggface)  // x0 = omega0 B^-1 r (cell blocks)
      launch_dg_bsmooth(c->dg, c->st, c->r, nullptr, c->dggface, c->mg_omega0, c->mgx, 0, s);
    else
      launch_mg_jacobi(n, c->st, c->r, nullptr, nullptr, c->dinv, c->mg_omega0, c->mgx, 0, s);
    mg_apply0(c, T, nullptr);
    HIPC(hipMemcpyAsync(z_dev, c->z, sizeof(double) * (size_t)n, hipMemcpyDeviceToDevice, s));
  }
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(s));
  return TV_OK;
}

}  // extern "C"
