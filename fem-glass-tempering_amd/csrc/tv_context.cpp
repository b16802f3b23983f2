// Context creation and destruction, mesh partition, device state and field
// transfer (reference interleaved layout <-> device component-major layout),
// time-series output and the Dirichlet setting.  C-ABI: include/tvfem.h.
//   tv_create            ThermoViscoProblem.__init__ (ThermoViscoProblem.py:24-58):
//                        spaces (:61-103), functions (:106-173)
//   tv_set_initial_condition  _set_initial_condition (:187-233)
//   tv_output_*          _write_initial_output / _write_output / _finalize
//                        (:246-276, :357-364, :614-620)
#include <cstdlib>

#include "tv_ctx.h"

namespace tv {

static std::mutex g_err_mu;
static std::string g_err;

void set_global_error(const std::string& m) {
  std::lock_guard<std::mutex> lk(g_err_mu);
  g_err = m;
}

// --------------------------------------------------------------------------------------
// geometry helpers
// --------------------------------------------------------------------------------------
void axis_coefs(const std::vector<double>& X, int first, int count, std::vector<double>& out) {
  // 1D P1 assembled mass / stiffness rows and adjacent cell lengths for global
  // nodes [first, first+count) of an axis with node coordinates X.
  const int n = (int)X.size();
  out.assign((size_t)count * C_NCOEF, 0.0);
  for (int q = 0; q < count; ++q) {
    const int i = first + q;
    double* c = &out[(size_t)q * C_NCOEF];
    if (n == 1) {
      c[C_MDI] = 1.0;
      continue;
    }
    const double hlo = (i > 0) ? X[i] - X[i - 1] : 0.0;
    const double hhi = (i < n - 1) ? X[i + 1] - X[i] : 0.0;
    c[C_MLO] = hlo / 6.0;
    c[C_MDI] = hlo / 3.0 + hhi / 3.0;
    c[C_MUP] = hhi / 6.0;
    c[C_KLO] = hlo > 0 ? -1.0 / hlo : 0.0;
    c[C_KDI] = (hlo > 0 ? 1.0 / hlo : 0.0) + (hhi > 0 ? 1.0 / hhi : 0.0);
    c[C_KUP] = hhi > 0 ? -1.0 / hhi : 0.0;
    c[C_HLO] = hlo;
    c[C_HHI] = hhi;
  }
}

const std::vector<double>& storage_coords(Ctx* c, int s, std::vector<double>& tmp) {
  if (c->perm[s] < 0) {
    tmp.assign(1, 0.0);
    return tmp;
  }
  return c->coords[c->perm[s]];
}

int alloc_field(Ctx* c, int id, int space, int bs) {
  FieldInfo& fi = c->f[id];
  fi.space = space;
  fi.bs = bs;
  const int64_t n = field_stride(c, space);
  // every field starts at its own offset inside a 2 MiB page (id x 132 KiB):
  // the fused visco update streams ~26 fields at the same index at once, and
  // page-aligned starts put all of them on the same HBM channels together
  const size_t stagger = (size_t)(id % 15) * (132u << 10);
  HIPC(hipMalloc(&fi.base, sizeof(double) * (size_t)std::max<int64_t>(1, n * bs) + stagger));
  fi.ptr = reinterpret_cast<double*>(static_cast<char*>(fi.base) + stagger);
  HIPC(hipMemsetAsync(fi.ptr, 0, sizeof(double) * (size_t)(n * bs), c->stream));
  fi.alloc = true;
  return TV_OK;
}

void alias_field(Ctx* c, int id, int target) {
  c->f[id] = c->f[target];
  c->f[id].alloc = false;
}

// storage axes: 0 = x (fastest); 2 = partition axis (slowest); 1 = the remaining
// axis (or degenerate).  Returns false for an invalid part_axis.
bool storage_perm(const tv_mesh_desc* m, int perm[3]) {
  const int d = m->dim;
  if (d == 1) {
    perm[0] = 0; perm[1] = -1; perm[2] = -1;
  } else if (d == 2) {
    perm[0] = 0; perm[1] = -1; perm[2] = 1;
  } else {
    int pa = m->part_axis;
    if (pa < 0) pa = (m->n_cells[1] >= m->n_cells[2]) ? 1 : 2;
    if (pa != 1 && pa != 2) return false;
    perm[0] = 0; perm[2] = pa; perm[1] = (pa == 1) ? 2 : 1;
  }
  return true;
}

// owned node planes [b0, b1) of partition p of P along the slowest storage axis
void part_planes(int N2, int P, int p, int* b0, int* b1) {
  *b0 = (int)((int64_t)N2 * p / P);
  *b1 = (int)((int64_t)N2 * (p + 1) / P);
}

// CG grid of `n2` local planes starting at global plane `first2` of storage
// axis 2 (ghost planes included: g_lo / g_hi of them), from the global node
// coordinates X[s] of the storage axes (a single 0 for a degenerate axis);
// bnd2lo / bnd2hi: the low / high face of axis 2 is a physical boundary here.
// Device arrays go to coef[3], *bnodes and ffbuf[2] (owned by the caller).
int build_cg_grid(Ctx* c, int d, const std::vector<double> (&X)[3], int first2, int n2, int g_lo, int g_hi,
                         bool bnd2lo, bool bnd2hi, CgGrid& g, double** coef, int64_t** bnodes, double** ffbuf) {
  g.n0 = (int)X[0].size();
  g.n1 = (int)X[1].size();
  g.g_lo = g_lo;
  g.g_hi = g_hi;
  g.n2 = n2;
  g.k_begin = g_lo;
  g.k_end = n2 - g_hi;
  g.w_begin = g.k_begin - std::max(0, g_lo - 1);
  g.w_end = g.k_end + std::max(0, g_hi - 1);
  g.deg1 = X[1].size() == 1;
  g.deg2 = X[2].size() == 1;
  g.bnd[0][0] = g.bnd[0][1] = 1;
  g.bnd[1][0] = g.bnd[1][1] = g.deg1 ? 0 : 1;
  g.bnd[2][0] = (!g.deg2 && bnd2lo) ? 1 : 0;
  g.bnd[2][1] = (!g.deg2 && bnd2hi) ? 1 : 0;
  const int first[3] = {0, 0, first2};
  const int cnt[3] = {g.n0, g.n1, g.n2};
  for (int s = 0; s < 3; ++s) {
    std::vector<double> cf;
    axis_coefs(X[s], first[s], cnt[s], cf);
    HIPC(hipMalloc(&coef[s], cf.size() * sizeof(double)));
    HIPC(hipMemcpy(coef[s], cf.data(), cf.size() * sizeof(double), hipMemcpyHostToDevice));
    g.coef[s] = coef[s];
  }
  const int64_t plane = (int64_t)g.n0 * g.n1;
  for (int f = 0; f < 6; ++f) g.ffoff[f] = -1;
  if (d == 3) {  // write-window nodes on physical boundary faces (Robin facets, marching kernel path)
    std::vector<int64_t> bn;
    for (int k = g.w_begin; k < g.w_end; ++k)
      for (int j = 0; j < g.n1; ++j)
        for (int i = 0; i < g.n0; ++i) {
          const bool on = (i == 0 && g.bnd[0][0]) || (i == g.n0 - 1 && g.bnd[0][1]) ||
                          (j == 0 && g.bnd[1][0]) || (j == g.n1 - 1 && g.bnd[1][1]) ||
                          (k == 0 && g.bnd[2][0]) || (k == g.n2 - 1 && g.bnd[2][1]);
          if (on) bn.push_back((int64_t)i + (int64_t)g.n0 * j + plane * k);
        }
    if (!bn.empty()) {
      HIPC(hipMalloc(bnodes, bn.size() * sizeof(int64_t)));
      HIPC(hipMemcpy(*bnodes, bn.data(), bn.size() * sizeof(int64_t), hipMemcpyHostToDevice));
    }
    g.bnodes = *bnodes;
    g.n_bnodes = (int64_t)bn.size();
    // facet-Jacobian terms: one value per node of every physical boundary
    // face, the six faces in one contiguous buffer, two parities
    const int nn[3] = {g.n0, g.n1, g.n2};
    int64_t tot = 0;
    for (int f = 0; f < 6; ++f) {
      const int ax = f >> 1, side = f & 1;
      g.fface[f] = nullptr;
      g.fn1[f] = g.fn2[f] = 0;
      g.ffoff[f] = -1;
      if (!g.bnd[ax][side]) continue;
      const int t1 = (ax == 0) ? 1 : 0, t2 = (ax == 2) ? 1 : 2;
      g.fn1[f] = nn[t1];
      g.fn2[f] = nn[t2];
      g.ffoff[f] = tot;
      tot += (int64_t)nn[t1] * nn[t2];
    }
    g.ffsize = tot;
    for (int q = 0; q < 2; ++q) {
      HIPC(hipMalloc(&ffbuf[q], sizeof(double) * (size_t)std::max<int64_t>(1, tot)));
      HIPC(hipMemsetAsync(ffbuf[q], 0, sizeof(double) * (size_t)std::max<int64_t>(1, tot), c->stream));
      g.ffbuf[q] = ffbuf[q];
    }
    for (int f = 0; f < 6; ++f) g.fface[f] = (g.ffoff[f] >= 0) ? ffbuf[0] + g.ffoff[f] : nullptr;
  }
  return TV_OK;
}

// Mixed families on a slab partition (the reference's main.py pairing DG T /
// CG sigma, ThermoViscoProblem.py:61-103 under mpiexec, and CG T / DG sigma).
// The T space is partitioned as on its own (CG: node planes [b0, b1) + one
// ghost plane per interface; DG: cell layers [b0, b1) + one ghost cell layer),
// the sigma space follows without ghosts of its own:
//  1 (DG T, CG sigma): sigma nodes on planes [b0, b1] are local -- [b0, b1)
//    owned, plane b1 too on the last part -- and node (i, j, k) reads the T dof
//    of the LAST cell fem::interpolate writes it from (the highest global cell
//    index around it: (min(i, C0-1), min(j, C1-1), min(k, C2-1))), which is an
//    owned cell, or for plane b1 of an inner part the ghost layer above;
//  2 (CG T, DG sigma): sigma owns the cell layers [b0, min(b1, C2)); every
//    corner node of those cells is local (plane b1 = the ghost plane above).
// The visco T pass runs over every local T dof (ghosts included: their T is
// exchanged after each Newton update, so they evolve as on their owners).
int setup_mixed_part(Ctx* c) {
  const int d = c->dim, nl = 1 << d;
  const int P = c->n_parts, p = c->part;
  const bool last = (p == P - 1);
  const int b0 = c->plane_begin, b1 = c->plane_end;
  const int C[3] = {std::max(1, c->Ncell_glob[0]), std::max(1, c->Ncell_glob[1]), std::max(1, c->Ncell_glob[2])};
  const int N0 = c->Nnode_glob[0], N1 = c->Nnode_glob[1];
  const bool act[3] = {true, c->perm[1] >= 0, c->perm[2] >= 0};
  const int64_t npl = (int64_t)N0 * N1;   // nodes per plane
  const int64_t pc = (int64_t)C[0] * C[1];  // cells per layer
  // local corner index l of a cell from the corner offsets (active axes only)
  auto corner = [&](const int bits[3]) {
    int l = 0, k = 0;
    for (int s = 0; s < 3; ++s) {
      if (!act[s]) continue;
      l |= bits[s] << k;
      ++k;
    }
    return l;
  };
  std::vector<int> map;
  if (c->fam_T == TV_DG) {  // 1: CG sigma on the nodes of planes [b0, b1]
    c->mixed_part = 1;
    const int nq = b1 - b0 + 1;
    c->nS = npl * nq;
    c->ownS_off = 0;
    c->ownS_n = npl * (last ? nq : nq - 1);
    c->globS_off = npl * b0;
    c->outS_n = c->nS;
    c->outT_n = c->ownT_n;
    const DgGrid& g = c->dg;
    map.assign((size_t)c->nS, -1);
    for (int k = b0; k <= b1; ++k)
      for (int j = 0; j < N1; ++j)
        for (int i = 0; i < N0; ++i) {
          const int ci[3] = {std::min(i, C[0] - 1), act[1] ? std::min(j, C[1] - 1) : 0,
                             act[2] ? std::min(k, C[2] - 1) : 0};
          const int bits[3] = {i - ci[0], j - ci[1], k - ci[2]};
          const int l = corner(bits);
          const int kl = ci[2] - b0 + g.k_begin;  // local cell layer
          int64_t base, stride;
          if (kl < g.k_begin) base = g.gofs[0], stride = pc;
          else if (kl >= g.k_end) base = g.gofs[1], stride = pc;
          else base = (int64_t)(kl - g.k_begin) * pc, stride = g.own;
          if (base < 0) return c->fail(TV_ERR_ARG, "mixed partition: a sigma node outside the local cells (internal)");
          const int64_t dof = base + (int64_t)l * stride + ci[0] + (int64_t)C[0] * ci[1];
          map[(size_t)(i + N0 * (j + (int64_t)N1 * (k - b0)))] = (int)dof;
        }
  } else {  // 2: DG sigma on the cell layers [b0, L1)
    c->mixed_part = 2;
    const int L1 = std::min(b1, C[2]);
    const int64_t ncl = pc * (L1 - b0);
    c->nS = ncl * nl;
    c->ownS_off = 0;
    c->ownS_n = c->nS;
    c->globS_off = pc * nl * b0;
    c->outS_n = c->nS;
    const CgGrid& g = c->cg;
    c->outT_n = c->ownT_n + (g.g_hi ? npl : 0);  // the plane above: the owned cells' upper corners
    map.assign((size_t)c->nS, -1);
    for (int64_t cl = 0; cl < ncl; ++cl) {
      const int ci[3] = {(int)(cl % C[0]), (int)((cl / C[0]) % C[1]), b0 + (int)(cl / pc)};
      for (int l = 0; l < nl; ++l) {
        int bits[3] = {0, 0, 0}, k = 0;
        for (int s = 0; s < 3; ++s) {
          if (!act[s]) continue;
          bits[s] = (l >> k) & 1;
          ++k;
        }
        const int kl = ci[2] + bits[2] - (b0 - g.g_lo);  // local node plane
        if (kl < 0 || kl >= g.n2) return c->fail(TV_ERR_ARG, "mixed partition: a corner outside the local planes (internal)");
        map[(size_t)((int64_t)l * ncl + cl)] =
            (int)((ci[0] + bits[0]) + (int64_t)g.n0 * ((ci[1] + bits[1]) + (int64_t)g.n1 * kl));
      }
    }
  }
  HIPC(hipMalloc(&c->map, sizeof(int) * (size_t)std::max<int64_t>(1, c->nS)));
  HIPC(hipMemcpy(c->map, map.data(), sizeof(int) * (size_t)c->nS, hipMemcpyHostToDevice));
  return TV_OK;
}

int setup_mesh(Ctx* c, const tv_mesh_desc* m) {
  const int d = m->dim;
  if (d < 1 || d > 3) return c->fail(TV_ERR_ARG, "mesh dim must be 1..3");
  c->dim = d;
  c->coords.resize(d);
  for (int a = 0; a < d; ++a) {
    if (m->n_cells[a] < 1) return c->fail(TV_ERR_ARG, "n_cells must be >= 1 on every axis");
    if (!m->coords[a]) return c->fail(TV_ERR_ARG, "coords missing");
    c->coords[a].assign(m->coords[a], m->coords[a] + m->n_cells[a] + 1);
    for (int i = 0; i < m->n_cells[a]; ++i)
      if (!(c->coords[a][i + 1] > c->coords[a][i]))
        return c->fail(TV_ERR_ARG, "node coordinates must be strictly increasing");
  }
  if (!storage_perm(m, c->perm)) return c->fail(TV_ERR_ARG, "part_axis must be 1 (y) or 2 (z) for 3D meshes");
  c->n_parts = std::max(1, m->n_parts);
  c->part = m->part;
  if (c->part < 0 || c->part >= c->n_parts) return c->fail(TV_ERR_ARG, "part out of range");
  if (c->n_parts > 1 && d == 1) return c->fail(TV_ERR_ARG, "partitioned meshes require dim >= 2");
  for (int s = 0; s < 3; ++s) {
    c->Ncell_glob[s] = (c->perm[s] < 0) ? 0 : m->n_cells[c->perm[s]];
    c->Nnode_glob[s] = c->Ncell_glob[s] + 1;
  }
  std::vector<double> tmp;
  if (c->fam_T == TV_CG) {
    const int N2 = c->Nnode_glob[2];
    const int P = c->n_parts, p = c->part;
    int b0, b1;
    part_planes(N2, P, p, &b0, &b1);
    if (b1 - b0 < 1) return c->fail(TV_ERR_ARG, "too many partitions for the mesh");
    c->plane_begin = b0;
    c->plane_end = b1;
    CgGrid& g = c->cg;
    std::vector<double> X[3];
    for (int s = 0; s < 3; ++s) X[s] = storage_coords(c, s, tmp);
    // deep ghosts (three planes per interface) for the distributed multigrid
    // with global coupling: the level-0 vectors of a V-cycle are then computed
    // on the ghost planes too and need no exchange of their own (tv_mgdist.cpp)
    // Every rank takes the same decision: from the SMALLEST slab of the global
    // partition (part_planes hands out sizes that differ by one plane), so a
    // partition too thin for deep ghosts gives every rank the one-ghost-plane
    // form instead of failing some ranks' creation while the others wait in
    // their first collective
    int min_slab = N2;
    for (int q = 0; q < P; ++q) {
      int q0, q1;
      part_planes(N2, P, q, &q0, &q1);
      min_slab = std::min(min_slab, q1 - q0);
    }
    // (an explicit SINGLE_REDUCTION with GMG is refused by mg_setup: the
    // single-reduction GMG-PCG is AUTO's choice on deep-ghost slabs)
    const bool deep = P > 1 && d == 3 && c->O.preconditioner == TV_PC_GMG && c->O.mg_coupling != TV_MG_COUPLING_LOCAL &&
                      min_slab >= kDeepGhosts;
    c->ghost_depth = deep ? kDeepGhosts : 1;
    const int G = c->ghost_depth;
    const int g_lo = (p > 0) ? G : 0, g_hi = (p < P - 1) ? G : 0;
    if (int e = build_cg_grid(c, d, X, b0 - g_lo, (b1 - b0) + g_lo + g_hi, g_lo, g_hi, p == 0, p == P - 1, g, c->coef,
                              &c->bnodes, c->ffbuf))
      return e;
    const int64_t plane = (int64_t)g.n0 * g.n1;
    c->nT = plane * g.n2;
    // the CG kernels index local nodes with 32-bit integers (68 M nodes = 290 GB
    // of state at materialize=1 would already exceed one MI355X)
    if (c->nT >= (int64_t)INT32_MAX) return c->fail(TV_ERR_ARG, "partition too large: >= 2^31 local nodes");
    c->ownT_off = plane * g.k_begin;
    c->ownT_n = plane * (g.k_end - g.k_begin);
    c->globT_off = plane * b0;
  } else {
    DgGrid& g = c->dg;
    g.c0 = c->Ncell_glob[0];
    g.c1 = std::max(1, c->Ncell_glob[1]);
    // partition: the owned cell layers [b0, b1) of storage axis 2 and one ghost
    // layer towards each neighbour (the SIPG facets of the interface)
    const int C2 = std::max(1, c->Ncell_glob[2]);
    const int P = c->n_parts, p = c->part;
    int b0 = 0, b1 = C2;
    if (P > 1) part_planes(C2, P, p, &b0, &b1);
    if (b1 - b0 < 1) return c->fail(TV_ERR_ARG, "too many partitions for the mesh");
    const int g_lo = (P > 1 && p > 0) ? 1 : 0, g_hi = (P > 1 && p < P - 1) ? 1 : 0;
    g.c2 = (b1 - b0) + g_lo + g_hi;
    g.k_begin = g_lo;
    g.k_end = g_lo + (b1 - b0);
    g.deg1 = (c->perm[1] < 0);
    g.deg2 = (c->perm[2] < 0);
    g.bnd[0][0] = g.bnd[0][1] = 1;
    g.bnd[1][0] = g.bnd[1][1] = g.deg1 ? 0 : 1;
    g.bnd[2][0] = (g.deg2 || p > 0) ? 0 : 1;
    g.bnd[2][1] = (g.deg2 || p < P - 1) ? 0 : 1;
    const int64_t pc = (int64_t)g.c0 * g.c1;
    const int nl0 = 1 << d;
    g.own = pc * (b1 - b0);
    g.gofs[0] = g_lo ? nl0 * g.own : -1;
    g.gofs[1] = g_hi ? nl0 * g.own + (int64_t)nl0 * pc * g_lo : -1;
    g.tile = c->O.dg_kernel == TV_DG_KERNEL_CELLS ? 0 : 1;  // 1: k_dg_tile with halo-loading edge waves
    g.tile_chunk = c->O.dg_tile_chunk > 0 ? c->O.dg_tile_chunk : 5;  // 5 planes measured best (C5)
    for (int s = 0; s < 3; ++s) {
      const std::vector<double>& X = storage_coords(c, s, tmp);
      std::vector<double> h;
      if (X.size() == 1) h.assign(1, 1.0);
      else if (s == 2) for (int k = b0 - g_lo; k < b1 + g_hi; ++k) h.push_back(X[k + 1] - X[k]);  // local layers
      else for (size_t i = 0; i + 1 < X.size(); ++i) h.push_back(X[i + 1] - X[i]);
      const size_t nh = h.size();
      for (size_t q = 0; q < nh; ++q) h.push_back(1.0 / h[q]);  // [h..., 1/h...]
      HIPC(hipMalloc(&c->dgh[s], h.size() * sizeof(double)));
      HIPC(hipMemcpy(c->dgh[s], h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
      g.h[s] = c->dgh[s];
      g.ih[s] = c->dgh[s] + nh;
    }
    const int nl = 1 << d;
    c->nT = (int64_t)g.c0 * g.c1 * g.c2 * nl;
    c->ownT_off = 0;              // the owned layers' dofs come first (DgGrid)
    c->ownT_n = g.own * nl;
    c->globT_off = (int64_t)b0 * pc * nl;  // cell-major global numbering: the owned cells are contiguous
    c->plane_begin = b0;
    c->plane_end = b1;
  }
  // sigma space
  if (c->fam_S == c->fam_T) {
    c->nS = c->nT;
    c->ownS_off = c->ownT_off;
    c->ownS_n = c->ownT_n;
    c->globS_off = c->globT_off;
  } else if (c->n_parts > 1) {
    if (int e = setup_mixed_part(c)) return e;
  } else {
    const int nl = 1 << d;
    const int64_t ncell = (int64_t)std::max(1, c->Ncell_glob[0]) * std::max(1, c->Ncell_glob[1]) *
                          std::max(1, c->Ncell_glob[2]);
    const int64_t nnode = (int64_t)c->Nnode_glob[0] * c->Nnode_glob[1] * c->Nnode_glob[2];
    c->nS = (c->fam_S == TV_CG) ? nnode : ncell * nl;
    c->ownS_off = 0;
    c->ownS_n = c->nS;
    c->globS_off = 0;
    // fem::interpolate: cells in order, last cell written wins at shared sigma dofs
    std::vector<int> map((size_t)c->nS, -1);
    const int C0 = std::max(1, c->Ncell_glob[0]), C1 = std::max(1, c->Ncell_glob[1]);
    const int N0 = c->Nnode_glob[0], N1 = c->Nnode_glob[1];
    const int act[3] = {0, c->perm[1] >= 0, c->perm[2] >= 0};
    for (int64_t cell = 0; cell < ncell; ++cell) {
      const int ci[3] = {(int)(cell % C0), (int)((cell / C0) % C1), (int)(cell / ((int64_t)C0 * C1))};
      for (int l = 0; l < nl; ++l) {
        int bits[3] = {0, 0, 0};
        int k = 0;
        for (int s = 0; s < 3; ++s) {
          if (s > 0 && !act[s]) continue;
          bits[s] = (l >> k) & 1;
          ++k;
        }
        const int64_t node = (int64_t)(ci[0] + bits[0]) + (int64_t)N0 * ((ci[1] + bits[1]) + (int64_t)N1 * (ci[2] + bits[2]));
        // DG dof numbering (cell-major) in device layout [l][cell]
        const int64_t dgdof = (int64_t)l * ncell + cell;
        if (c->fam_S == TV_CG) map[(size_t)node] = (int)dgdof;  // sigma CG <- T DG
        else map[(size_t)dgdof] = (int)node;                    // sigma DG <- T CG
      }
    }
    HIPC(hipMalloc(&c->map, sizeof(int) * (size_t)c->nS));
    HIPC(hipMemcpy(c->map, map.data(), sizeof(int) * (size_t)c->nS, hipMemcpyHostToDevice));
  }
  // thermal constants
  const tv_params& P = c->P;
  for (CgGrid* g = &c->cg; g; g = nullptr) {
    g->dt = P.dt; g->dt_alpha = P.dt * P.alpha; g->dt_f = P.dt * P.f;
    g->a_rad = 0.001 * (P.sigma * P.epsilon); g->a_conv = 0.001 * P.htc;
    g->T_amb = P.T_ambient; g->T_amb4 = P.T_ambient * P.T_ambient * P.T_ambient * P.T_ambient;
  }
  {
    DgGrid* g = &c->dg;
    g->dt = P.dt; g->dt_alpha = P.dt * P.alpha; g->dt_f = P.dt * P.f;
    g->a_rad = 0.001 * (P.sigma * P.epsilon); g->a_conv = 0.001 * P.htc;
    g->T_amb = P.T_ambient; g->T_amb4 = P.T_ambient * P.T_ambient * P.T_ambient * P.T_ambient;
    g->penalty = 5.0;
  }
  return TV_OK;
}


int setup_fields(Ctx* c) {
  const int d = c->dim, dd = d * d;
  const bool all = c->O.materialize != 0;
  int rc;
#define AF(id, sp, bs) if ((rc = alloc_field(c, id, sp, bs)) != TV_OK) return rc
  AF(TV_F_T, 0, 1);
  AF(TV_F_T_PREV, 0, 1);
  AF(TV_F_TF, 0, 1);
  AF(TV_F_TF_PARTIAL, 0, 6);
  AF(TV_F_PHI, 0, 1);
  AF(TV_F_XI, 0, 1);
  AF(TV_F_S_TILDE, 1, 6 * dd);
  AF(TV_F_SIGMA_TILDE, 1, 6 * dd);
  AF(TV_F_SIGMA, 1, dd);
  const bool paper = c->O.model_mode == TV_MODEL_PAPER;
  if (paper && !all) {  // s / sigma partial feed s~ / sigma~ (Eq. 16): state in paper mode
    AF(TV_F_S_PARTIAL, 1, 6 * dd);
    AF(TV_F_SIGMA_PARTIAL, 1, 6 * dd);
    alias_field(c, TV_F_S_PARTIAL_NEXT, TV_F_S_PARTIAL);
    alias_field(c, TV_F_SIGMA_PARTIAL_NEXT, TV_F_SIGMA_PARTIAL);
  }
  if (paper && c->fam_T != c->fam_S) HIPC(hipMalloc(&c->Tfo, sizeof(double) * (size_t)std::max<int64_t>(1, c->nT)));
  if (all) {
    AF(TV_F_T_NEXT, 0, 1);
    AF(TV_F_PHI_NEXT, 0, 1);
    AF(TV_F_THERMAL_STRAIN, 1, dd);
    AF(TV_F_TOTAL_STRAIN, 1, dd);
    AF(TV_F_DEVIATORIC_STRAIN, 1, dd);
    AF(TV_F_DS_PARTIAL, 1, 6 * dd);
    AF(TV_F_DSIGMA_PARTIAL, 1, 6 * dd);
    AF(TV_F_S_PARTIAL, 1, 6 * dd);
    AF(TV_F_SIGMA_PARTIAL, 1, 6 * dd);
    alias_field(c, TV_F_S_PARTIAL_NEXT, TV_F_S_PARTIAL);
    alias_field(c, TV_F_SIGMA_PARTIAL_NEXT, TV_F_SIGMA_PARTIAL);
  }
#undef AF
  alias_field(c, TV_F_TF_PREV, TV_F_TF);
  alias_field(c, TV_F_TF_PARTIAL_PREV, TV_F_TF_PARTIAL);
  alias_field(c, TV_F_S_TILDE_NEXT, TV_F_S_TILDE);
  alias_field(c, TV_F_SIGMA_TILDE_NEXT, TV_F_SIGMA_TILDE);
  // PCG work vectors (T space, local size)
  const size_t nb = sizeof(double) * (size_t)std::max<int64_t>(1, c->nT);
  HIPC(hipMalloc(&c->r, nb));
  HIPC(hipMalloc(&c->z, nb));
  HIPC(hipMalloc(&c->pA, nb));
  HIPC(hipMalloc(&c->pB, nb));
  HIPC(hipMalloc(&c->w, nb));
  HIPC(hipMalloc(&c->dinv, nb));
  for (double* p : {c->r, c->z, c->pA, c->pB, c->w, c->dinv}) HIPC(hipMemsetAsync(p, 0, nb, c->stream));
  c->f[TV_F_RESIDUAL].ptr = c->r; c->f[TV_F_RESIDUAL].bs = 1; c->f[TV_F_RESIDUAL].space = 0;
  if (int e = alloc_field(c, TV_F_DX, 0, 1)) return e;
  int np = kVecBlocksMax;
  if (c->um) np = std::max(np, um_num_blocks(c->umg));
  else if (c->fam_T == TV_CG) np = std::max(np, cg_num_blocks(c->cg, true));
  else np = std::max(np, dg_num_blocks(c->dg));
  c->n_partials_cap = np;
  // records of width <= 3 per workgroup + the shard records of the two-level tail
  HIPC(hipMalloc(&c->partials, sizeof(double) * 3 * ((size_t)np + 2 * kShards)));
  HIPC(hipMalloc(&c->sums, sizeof(double) * 8));
  HIPC(hipMalloc(&c->ngate, sizeof(double) * 8));
  HIPC(hipMemset(c->ngate, 0, sizeof(double) * 8));
  if (const char* e = std::getenv("TVFEM_NEWTON_AHEAD")) c->newton_ahead = std::atoi(e) != 0;
  HIPC(hipMalloc(&c->counters, sizeof(unsigned) * kCounterWords));
  HIPC(hipMemsetAsync(c->counters, 0, sizeof(unsigned) * kCounterWords, c->stream));
  HIPC(hipMalloc(&c->st, sizeof(PcgState)));
  HIPC(hipMalloc(&c->tflag, sizeof(int)));
  HIPC(hipMemsetAsync(c->tflag, 0, sizeof(int), c->stream));  // the tilde fields start at +0.0
  HIPC(hipHostMalloc(&c->h_st, 3 * sizeof(PcgState)));
  for (int k = 0; k < 2; ++k) HIPC(hipEventCreateWithFlags(&c->evp[k], hipEventDisableTiming));
  for (hipEvent_t& e : c->evn) HIPC(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIPC(hipHostMalloc(&c->h_sums, sizeof(double) * 8));
  const int var = c->O.pcg_variant;
  const bool can = c->fam_T == TV_CG && !c->um && cg_cgs_supported(c->cg);
  if (var == TV_PCG_SINGLE_REDUCTION && !can)
    return c->fail(TV_ERR_ARG, "pcg_variant SINGLE_REDUCTION needs a 3D CG1 temperature space");
  // AUTO: the single-reduction form where the mesh is partitioned into slabs
  // of at most kCgsAutoMaxNodes owned nodes (one RCCL group per iteration
  // instead of two all-reduces + a halo + two logic launches), and on one
  // partition of at most kCgsAutoMaxNodes1 nodes, where an iteration is
  // launch-latency bound and one launch beats two (round 3, one box, same
  // Krylov counts: C3 1.05M nodes 2.97 vs 3.14 ms/step, C2 112K nodes 1.02-1.05
  // vs 1.06 ms; profiles/r03_single_reduction_c2_c3.txt); on larger grids its
  // heavier launch is bandwidth-bound and KSPCG's two lighter launches are
  // faster (measured on the C4 per-rank shares, DESIGN.md §5: 4.1M nodes 13.2
  // vs 18.3 ms/step, against ~2.7 ms of communication the single reduction
  // saves; 2M nodes 7.6 vs 8.6 ms)
  // The choice must agree on every rank (the two forms issue different
  // collectives): it is taken on the LARGEST slab of the partition, which every
  // rank computes identically from the global mesh, not on this rank's own slab
  // (slabs differ by a plane, so ranks could fall on both sides of the bound)
  int64_t max_slab = c->ownT_n;
  if (c->n_parts > 1 && c->fam_T == TV_CG && !c->um) {
    const int64_t plane = (int64_t)c->Nnode_glob[0] * c->Nnode_glob[1];
    for (int p = 0; p < c->n_parts; ++p) {
      int b0, b1;
      part_planes(c->Nnode_glob[2], c->n_parts, p, &b0, &b1);
      max_slab = std::max<int64_t>(max_slab, plane * (b1 - b0));
    }
  }
  c->cgs = can && (var == TV_PCG_SINGLE_REDUCTION ||
                   (var == TV_PCG_AUTO &&
                    (c->n_parts > 1 ? max_slab <= kCgsAutoMaxNodes : c->nT <= kCgsAutoMaxNodes1) &&
                    c->O.preconditioner != TV_PC_GMG));  // the multigrid solve runs in the KSPCG form
  if (c->cgs) {
    for (double** q : {&c->cr[0], &c->cr[1], &c->cs[0], &c->cs[1], &c->cw1}) {
      HIPC(hipMalloc(q, nb));
      HIPC(hipMemsetAsync(*q, 0, nb, c->stream));
    }
    const size_t plane = (size_t)c->cg.n0 * c->cg.n1;
    HIPC(hipMalloc(&c->wsend, sizeof(double) * 2 * plane));
  }
  return TV_OK;
}

// --------------------------------------------------------------------------------------
// field transfer: reference interleaved layout <-> device component-major layout
// --------------------------------------------------------------------------------------
__global__ void k_interleave(int dir, double* __restrict__ buf, double* __restrict__ dev, int64_t ndof, int bs,
                             int64_t stride, int64_t off, int dg_nl, int64_t dg_ncell) {
  // dir 0: buf (host layout, dof*bs+comp) -> dev ; dir 1: dev -> buf
  const int64_t total = ndof * bs;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t dof = t / bs;
    const int comp = (int)(t % bs);
    int64_t di = (dg_nl > 0) ? (dof % dg_nl) * dg_ncell + dof / dg_nl : off + dof;
    double* p = dev + comp * stride + di;
    if (dir == 0) *p = buf[t];
    else buf[t] = *p;
  }
}

int transfer(Ctx* c, int field, double* host, size_t n, int dir) {
  if (field < 0 || field >= TV_NUM_FIELDS) return c->fail(TV_ERR_ARG, "bad field id");
  FieldInfo& fi = c->f[field];
  if (!fi.ptr) return c->fail(TV_ERR_STATE, "field not materialized (options.materialize = 0 keeps state fields only)");
  const int64_t ndof = (fi.space == 0) ? c->ownT_n : c->ownS_n;
  const int64_t off = (fi.space == 0) ? c->ownT_off : c->ownS_off;
  const int64_t stride = field_stride(c, fi.space);
  const size_t need = (size_t)ndof * fi.bs;
  if (n != need)
    return c->fail(TV_ERR_ARG, "size mismatch: expected " + std::to_string(need) + " values, got " + std::to_string(n));
  const bool dgsp = (fi.space == 0 ? c->fam_T : c->fam_S) == TV_DG;
  const int nl = dgsp ? (1 << c->dim) : 0;
  const int64_t ncell = dgsp ? ndof / nl : 0;
  const size_t bytes = need * sizeof(double);
  if (c->scratch_bytes < bytes) {
    if (c->scratch) HIPC(hipFree(c->scratch));
    c->scratch = nullptr;
    HIPC(hipMalloc(&c->scratch, std::max<size_t>(bytes, 8)));
    c->scratch_bytes = bytes;
  }
  const int blocks = (int)std::min<int64_t>(std::max<int64_t>(1, ((int64_t)need + 255) / 256), 16384);
  if (dir == 0) {
    if (((c->um && c->n_parts > 1) || (c->mixed_part && fi.space == 0)) && field != TV_F_T && field != TV_F_T_PREV)
      c->ghost_dirty |= 1u << field;
    const bool tilde = field == TV_F_S_TILDE || field == TV_F_S_TILDE_NEXT || field == TV_F_SIGMA_TILDE ||
                       field == TV_F_SIGMA_TILDE_NEXT;
    if (tilde) {  // values other than +0.0 end the all-zero tracking of the tilde fields
      const uint64_t* b = reinterpret_cast<const uint64_t*>(host);
      uint64_t any = 0;
      for (size_t k = 0; k < need; ++k) any |= b[k];
      if (any) {
        static const int one = 1;
        HIPC(hipMemcpyAsync(c->tflag, &one, sizeof(int), hipMemcpyHostToDevice, c->stream));
      }
    }
    HIPC(hipMemcpyAsync(c->scratch, host, bytes, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(k_interleave, dim3(blocks), dim3(256), 0, c->stream, 0, c->scratch, fi.ptr, ndof, fi.bs,
                       stride, off, nl, ncell);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(c->stream));
  } else {
    hipLaunchKernelGGL(k_interleave, dim3(blocks), dim3(256), 0, c->stream, 1, c->scratch, fi.ptr, ndof, fi.bs,
                       stride, off, nl, ncell);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(host, c->scratch, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
  }
  return TV_OK;
}

}  // namespace tv

using namespace tv;

extern "C" {

int tv_abi_version(void) { return TV_ABI_VERSION; }


const char* tv_last_error(const void* ctx) {
  if (ctx) return static_cast<const Ctx*>(ctx)->err.c_str();
  std::lock_guard<std::mutex> lk(g_err_mu);
  return g_err.c_str();
}


void tv_default_options(tv_options* o) {
  o->newton_rtol = 1e-12;  // ThermoViscoProblem.py:336
  o->newton_atol = 1e-10;  // dolfinx NewtonSolver default
  o->newton_max_it = 50;   // dolfinx default
  o->error_on_nonconvergence = 1;
  o->ksp_rtol = 1e-5;      // PETSc defaults
  o->ksp_atol = 1e-50;
  o->ksp_dtol = 1e5;
  o->ksp_max_it = 10000;
  o->materialize = 1;
  o->pcg_batch = 8;
  o->pcg_variant = TV_PCG_AUTO;
  o->model_mode = TV_MODEL_REFERENCE;
  o->preconditioner = TV_PC_JACOBI;
  o->mg_levels = 0;
  o->dg_kernel = TV_DG_KERNEL_AUTO;
  o->dg_tile_chunk = 0;
  o->mg_replicate_nodes = 0;
  o->ksp_fixed_its = 0;
  o->mg_coupling = TV_MG_COUPLING_AUTO;
}


void tv_default_params(tv_params* p) {
  std::memset(p, 0, sizeof(*p));
  // main.py:29-55
  p->f = 0.0; p->epsilon = 0.93; p->sigma = 5.670e-8; p->T_ambient = 600.0; p->T_0 = 800.0;
  p->alpha = 1.0; p->htc = 280.1; p->rho = 2500.0; p->cp = 1433.0; p->k = 1.0;
  p->H = 627.8e3; p->Tb = 869.0; p->Rg = 8.314; p->alpha_solid = 9.10e-6; p->alpha_liquid = 25.10e-6;
  p->Tf_init = 873.0;
  // ViscoelasticModel.py:19-68
  const double m[6] = {5.523e-2, 8.205e-2, 1.215e-1, 2.286e-1, 2.860e-1, 2.265e-1};
  const double lm[6] = {5.965e-4, 1.077e-2, 1.362e-1, 1.505e-1, 6.747e+0, 2.963e+1};
  const double g[6] = {1.585, 2.354, 3.486, 6.558, 8.205, 6.498};
  const double lg[6] = {6.658e-5, 1.197e-3, 1.514e-2, 1.672e-1, 7.497e-1, 3.292e+0};
  const double k[6] = {7.588e-1, 7.650e-1, 9.806e-1, 7.301e+0, 1.347e+1, 1.090e+1};
  const double lk[6] = {5.009e-5, 9.945e-4, 2.022e-3, 1.925e-2, 1.199e-1, 2.033e+0};
  for (int i = 0; i < 6; ++i) {
    p->m_n[i] = m[i]; p->lambda_m[i] = lm[i]; p->g_n[i] = g[i];
    p->lambda_g[i] = lg[i]; p->k_n[i] = k[i]; p->lambda_k[i] = lk[i];
  }
  p->dt = 0.1;  // main.py:16
}


int tv_create(const tv_mesh_desc* mesh, const tv_fe_config* fe, const tv_params* params, const tv_options* opts,
              int device, void** ctx_out) {
  if (!mesh || !fe || !params || !ctx_out) {
    set_global_error("tv_create: null argument");
    return TV_ERR_ARG;
  }
  *ctx_out = nullptr;
  auto c = std::make_unique<Ctx>();
  if (fe->T_degree != 1 || fe->sigma_degree != 1) {
    set_global_error("only degree-1 Lagrange elements are implemented");
    return TV_ERR_ARG;
  }
  if ((fe->T_family != TV_CG && fe->T_family != TV_DG) || (fe->sigma_family != TV_CG && fe->sigma_family != TV_DG)) {
    set_global_error("Only CG and DG elements are supported");
    return TV_ERR_ARG;
  }
  if (!(params->dt > 0.0)) {
    set_global_error("dt must be positive");
    return TV_ERR_ARG;
  }
  c->fam_T = fe->T_family;
  c->fam_S = fe->sigma_family;
  c->P = *params;
  if (opts) c->O = *opts;
  else tv_default_options(&c->O);
  c->device = device;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    set_global_error("no HIP device available: libtvfem requires an MI355X (gfx950) GPU");
    return TV_ERR_HIP;
  }
  if (device < 0 || device >= ndev) {
    set_global_error("device index out of range");
    return TV_ERR_ARG;
  }
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
    set_global_error("HIP stream/event creation failed");
    return TV_ERR_HIP;
  }
  if (c->O.preconditioner == TV_PC_AMG) {
    set_global_error("TV_PC_AMG: unstructured meshes (the box meshes take TV_PC_GMG)");
    return TV_ERR_ARG;
  }
  int rc = setup_mesh(c.get(), mesh);
  if (rc == TV_OK) rc = setup_fields(c.get());
  if (rc == TV_OK && c->O.preconditioner == TV_PC_GMG) rc = mg_setup(c.get());
  else if (rc == TV_OK && c->O.preconditioner != TV_PC_JACOBI) rc = c->fail(TV_ERR_ARG, "unknown preconditioner");
  if (rc == TV_OK && hipStreamSynchronize(c->stream) != hipSuccess) rc = c->fail(TV_ERR_HIP, "sync failed");
  if (rc != TV_OK) {
    set_global_error(c->err);
    tv_destroy(c.release());
    return rc;
  }
  *ctx_out = c.release();
  return TV_OK;
}


static int setup_umesh(Ctx* c, const tv_umesh_desc* m, const tv_upart_desc* pd) {
  const int d = m->dim;
  if (d != 2 && d != 3) return c->fail(TV_ERR_ARG, "unstructured meshes: dim 2 (quadrilaterals) or 3 (hexahedra)");
  if (c->fam_T != TV_CG || c->fam_S != TV_CG)
    return c->fail(TV_ERR_ARG, "unstructured meshes: CG temperature and stress spaces only");
  if (m->n_vertices < 1 || m->n_cells < 1 || !m->coords || !m->cells) return c->fail(TV_ERR_ARG, "empty mesh");
  if (m->n_vertices >= INT32_MAX) return c->fail(TV_ERR_ARG, "unstructured meshes: < 2^31 vertices");
  const int nl = 1 << d;
  for (int64_t k = 0; k < m->n_cells * nl; ++k)
    if (m->cells[k] < 0 || m->cells[k] >= m->n_vertices) return c->fail(TV_ERR_ARG, "cell vertex index out of range");
  int64_t nown = m->n_vertices;
  if (pd) {  // the partition's communication plan (tv_upart_desc)
    if (pd->n_parts < 1 || pd->part < 0 || pd->part >= pd->n_parts || pd->n_owned < 1 ||
        pd->n_owned > m->n_vertices || pd->n_owned_cells < 1 || pd->n_owned_cells > m->n_cells ||
        pd->global_offset < 0 || pd->n_neighbors < 0 || pd->n_neighbors >= pd->n_parts ||
        (pd->n_neighbors > 0 && (!pd->neighbors || !pd->recv_count || !pd->send_count)))
      return c->fail(TV_ERR_ARG, "tv_upart_desc: inconsistent partition description");
    nown = pd->n_owned;
    int64_t rt = 0, stot = 0;
    for (int k = 0; k < pd->n_neighbors; ++k) {
      const int q = pd->neighbors[k];
      if (q < 0 || q >= pd->n_parts || q == pd->part || (k > 0 && q <= pd->neighbors[k - 1]) ||
          pd->recv_count[k] < 0 || pd->send_count[k] < 0)
        return c->fail(TV_ERR_ARG, "tv_upart_desc: neighbours must be distinct ascending ranks other than part");
      c->um_peer.push_back(q);
      c->um_rcnt.push_back(pd->recv_count[k]);
      c->um_roff.push_back(rt);
      c->um_scnt.push_back(pd->send_count[k]);
      c->um_soff.push_back(stot);
      rt += pd->recv_count[k];
      stot += pd->send_count[k];
    }
    if (nown + rt != m->n_vertices) return c->fail(TV_ERR_ARG, "tv_upart_desc: n_owned + received ghosts != vertices");
    if (stot > 0 && !pd->send_idx) return c->fail(TV_ERR_ARG, "tv_upart_desc: send_idx missing");
    for (int64_t k = 0; k < stot; ++k)
      if (pd->send_idx[k] < 0 || pd->send_idx[k] >= nown)
        return c->fail(TV_ERR_ARG, "tv_upart_desc: send_idx must name owned vertices");
    if (stot > 0) {
      HIPC(hipMalloc(&c->um_sidx, sizeof(int64_t) * (size_t)stot));
      HIPC(hipMemcpy(c->um_sidx, pd->send_idx, sizeof(int64_t) * (size_t)stot, hipMemcpyHostToDevice));
      HIPC(hipMalloc(&c->um_sbuf, sizeof(double) * (size_t)stot));
    }
    c->n_parts = pd->n_parts;
    c->part = pd->part;
    c->um_own_cells = pd->n_owned_cells;
  } else {
    c->um_own_cells = m->n_cells;
  }
  c->um = true;
  c->dim = d;
  c->um_xyz.assign(m->coords, m->coords + 3 * m->n_vertices);
  c->um_cells.assign(m->cells, m->cells + m->n_cells * nl);
  const tv_params& P = c->P;
  UmGrid& g = c->umg;
  g.dt = P.dt; g.dt_alpha = P.dt * P.alpha; g.dt_f = P.dt * P.f;
  g.a_rad = 0.001 * (P.sigma * P.epsilon); g.a_conv = 0.001 * P.htc;
  g.T_amb = P.T_ambient; g.T_amb4 = P.T_ambient * P.T_ambient * P.T_ambient * P.T_ambient;
  std::string err;
  if (um_setup(d, m->n_vertices, nown, m->coords, m->n_cells, m->cells, g, c->umd, c->stream, err) != 0)
    return c->fail(err.rfind("HIP", 0) == 0 ? TV_ERR_HIP : TV_ERR_ARG, err);
  std::vector<unsigned char> bm;
  um_boundary_vertices(c->umd, bm);
  HIPC(hipMalloc(&c->um_bmask, bm.size()));
  HIPC(hipMemcpy(c->um_bmask, bm.data(), bm.size(), hipMemcpyHostToDevice));
  c->nT = c->nS = g.nv;
  c->ownT_off = c->ownS_off = 0;
  c->ownT_n = c->ownS_n = nown;
  c->globT_off = c->globS_off = pd ? pd->global_offset : 0;
  return TV_OK;
}


static int create_unstructured(const tv_umesh_desc* mesh, const tv_upart_desc* part, const tv_fe_config* fe,
                               const tv_params* params, const tv_options* opts, int device, void** ctx_out) {
  if (!mesh || !fe || !params || !ctx_out) {
    set_global_error("tv_create_unstructured: null argument");
    return TV_ERR_ARG;
  }
  *ctx_out = nullptr;
  auto c = std::make_unique<Ctx>();
  if (fe->T_degree != 1 || fe->sigma_degree != 1) {
    set_global_error("only degree-1 Lagrange elements are implemented");
    return TV_ERR_ARG;
  }
  if (!(params->dt > 0.0)) {
    set_global_error("dt must be positive");
    return TV_ERR_ARG;
  }
  c->fam_T = fe->T_family;
  c->fam_S = fe->sigma_family;
  c->P = *params;
  if (opts) c->O = *opts;
  else tv_default_options(&c->O);
  c->device = device;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    set_global_error("no HIP device available: libtvfem requires an MI355X (gfx950) GPU");
    return TV_ERR_HIP;
  }
  if (device < 0 || device >= ndev) {
    set_global_error("device index out of range");
    return TV_ERR_ARG;
  }
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
    set_global_error("HIP stream/event creation failed");
    return TV_ERR_HIP;
  }
  if (c->O.preconditioner != TV_PC_JACOBI && c->O.preconditioner != TV_PC_AMG) {
    set_global_error("unstructured meshes: preconditioner TV_PC_JACOBI or TV_PC_AMG (the box multigrid needs a "
                     "rectilinear mesh)");
    return TV_ERR_ARG;
  }
  int rc = setup_umesh(c.get(), mesh, part);
  if (rc == TV_OK) rc = setup_fields(c.get());
  // a partition builds its (agglomerated) hierarchy at its first solve: the
  // setup gathers the global operator through the communicator set after creation
  if (rc == TV_OK && c->O.preconditioner == TV_PC_AMG && c->n_parts < 2) rc = amg_setup(c.get());
  if (rc == TV_OK && hipStreamSynchronize(c->stream) != hipSuccess) rc = c->fail(TV_ERR_HIP, "sync failed");
  if (rc != TV_OK) {
    set_global_error(c->err);
    tv_destroy(c.release());
    return rc;
  }
  *ctx_out = c.release();
  return TV_OK;
}


int tv_create_unstructured(const tv_umesh_desc* mesh, const tv_fe_config* fe, const tv_params* params,
                           const tv_options* opts, int device, void** ctx_out) {
  return create_unstructured(mesh, nullptr, fe, params, opts, device, ctx_out);
}


int tv_create_unstructured_part(const tv_umesh_desc* local_mesh, const tv_upart_desc* part, const tv_fe_config* fe,
                                const tv_params* params, const tv_options* opts, int device, void** ctx_out) {
  if (!part) {
    set_global_error("tv_create_unstructured_part: null partition description");
    return TV_ERR_ARG;
  }
  return create_unstructured(local_mesh, part, fe, params, opts, device, ctx_out);
}


int tv_partition_rcb(const tv_umesh_desc* m, int n_parts, int* part_out) {
  if (!m || !part_out || !m->coords || !m->cells || (m->dim != 2 && m->dim != 3)) {
    set_global_error("tv_partition_rcb: bad argument");
    return TV_ERR_ARG;
  }
  std::string err;
  if (um_rcb(m->dim, m->n_vertices, m->coords, m->n_cells, m->cells, n_parts, part_out, err)) {
    set_global_error(err);
    return TV_ERR_ARG;
  }
  return TV_OK;
}


int tv_partition_layout(const tv_mesh_desc* m, int64_t* out) {
  if (!m || !out || m->dim < 1 || m->dim > 3 || m->n_parts < 1 || m->part < 0 || m->part >= m->n_parts) {
    set_global_error("tv_partition_layout: invalid arguments");
    return TV_ERR_ARG;
  }
  int perm[3];
  if (!storage_perm(m, perm)) {
    set_global_error("part_axis must be 1 (y) or 2 (z) for 3D meshes");
    return TV_ERR_ARG;
  }
  int N[3];
  for (int s = 0; s < 3; ++s) N[s] = (perm[s] < 0) ? 1 : m->n_cells[perm[s]] + 1;
  int b0, b1;
  part_planes(N[2], m->n_parts, m->part, &b0, &b1);
  const int64_t plane = (int64_t)N[0] * N[1];
  const int glo = m->part > 0, ghi = m->part < m->n_parts - 1;
  out[0] = perm[0]; out[1] = perm[1]; out[2] = perm[2];
  out[3] = N[0]; out[4] = N[1]; out[5] = N[2];
  out[6] = b0; out[7] = b1;
  out[8] = plane * b0;                          // global offset of the first owned dof
  out[9] = plane * (b1 - b0);                   // owned dofs
  out[10] = plane * ((b1 - b0) + glo + ghi);   // local dofs (owned + ghost planes)
  out[11] = glo; out[12] = ghi;
  return TV_OK;
}


int tv_destroy(void* ctx) {
  if (!ctx) return TV_OK;
  Ctx* c = static_cast<Ctx*>(ctx);
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->out) output_destroy(c->out);
  for (int i = 0; i < TV_NUM_FIELDS; ++i)
    if (c->f[i].alloc && c->f[i].base) hipFree(c->f[i].base);
  for (double* p : {c->cr[0], c->cr[1], c->cs[0], c->cs[1], c->cw1, c->wsend, c->dB, c->dtmp, c->Tfo})
    if (p) hipFree(p);
  um_free(c->umd);
  if (c->um_bmask) hipFree(c->um_bmask);
  if (c->um_sidx) hipFree(c->um_sidx);
  for (void* p : c->amg_bufs) hipFree(p);
  if (c->um_sbuf) hipFree(c->um_sbuf);
  for (MgLevel& L : c->mg) {
    for (void* p : L.bufs) hipFree(p);
    for (int s = 0; s < 3; ++s)
      if (L.coef[s]) hipFree(L.coef[s]);
    if (L.bnodes) hipFree(L.bnodes);
    for (int q = 0; q < 2; ++q)
      if (L.ffbuf[q]) hipFree(L.ffbuf[q]);
    if (L.mask) hipFree(L.mask);
  }
  if (c->mgx) hipFree(c->mgx);
  if (c->mg_s) hipFree(c->mg_s);
  if (c->dggface) hipFree(c->dggface);
  for (double* p : {c->r, c->z, c->pA, c->pB, c->w, c->dinv, c->partials, c->sums, c->ngate, c->scratch})
    if (p) hipFree(p);
  for (int s = 0; s < 3; ++s) {
    if (c->coef[s]) hipFree(c->coef[s]);
    if (c->dgh[s]) hipFree(c->dgh[s]);
  }
  if (c->map) hipFree(c->map);
  if (c->bnodes) hipFree(c->bnodes);
  for (int q = 0; q < 2; ++q)
    if (c->ffbuf[q]) hipFree(c->ffbuf[q]);
  if (c->st) hipFree(c->st);
  if (c->tflag) hipFree(c->tflag);
  if (c->counters) hipFree(c->counters);
  if (c->h_st) hipHostFree(c->h_st);
  if (c->h_sums) hipHostFree(c->h_sums);
  if (c->d_dirty) hipFree(c->d_dirty);
  if (c->dg_sbuf) hipFree(c->dg_sbuf);
  if (c->h_halo) hipHostFree(c->h_halo);
  if (c->h_big) hipHostFree(c->h_big);
  if (c->mg_mask0) hipFree(c->mg_mask0);
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->ev0) hipEventDestroy(c->ev0);
  if (c->ev1) hipEventDestroy(c->ev1);
  for (int k = 0; k < 2; ++k) {
    if (c->evp[k]) hipEventDestroy(c->evp[k]);
    if (c->vev[k]) hipEventDestroy(c->vev[k]);
  }
  for (hipEvent_t e : c->evn)
    if (e) hipEventDestroy(e);
  if (c->d_ts) hipFree(c->d_ts);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
  return TV_OK;
}


int tv_num_dofs(void* ctx, int space, int64_t* n_owned, int64_t* global_offset) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  if (n_owned) *n_owned = space == 0 ? c->ownT_n : c->ownS_n;
  if (global_offset) *global_offset = space == 0 ? c->globT_off : c->globS_off;
  return TV_OK;
}


int tv_field_block_size(void* ctx, int field, int* bs) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || field < 0 || field >= TV_NUM_FIELDS) return TV_ERR_ARG;
  const int dd = c->dim * c->dim;
  static const int kind[TV_NUM_FIELDS] = {1, 1, 1, 1, 1, 6, 6, 1, 1, 1, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3, 3, 3, 2, 1, 1};
  const int k = kind[field];
  *bs = (k == 1) ? 1 : (k == 6 ? 6 : (k == 2 ? dd : 6 * dd));
  return TV_OK;
}


int tv_dof_coordinates(void* ctx, int space, double* xyz, size_t n_dofs) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !xyz) return TV_ERR_ARG;
  const int fam = space == 0 ? c->fam_T : c->fam_S;
  const int64_t nown = space == 0 ? c->ownT_n : c->ownS_n;
  if ((int64_t)n_dofs != nown) return c->fail(TV_ERR_ARG, "n_dofs mismatch");
  if (c->um) {
    std::memcpy(xyz, c->um_xyz.data(), sizeof(double) * 3 * (size_t)nown);
    return TV_OK;
  }
  std::vector<double> tmp;
  const std::vector<double>* X[3];
  std::vector<double> deg(1, 0.0);
  for (int s = 0; s < 3; ++s) X[s] = (c->perm[s] < 0) ? &deg : &c->coords[c->perm[s]];
  const int N0 = c->Nnode_glob[0], N1 = c->Nnode_glob[1];
  if (fam == TV_CG) {
    const int64_t base = (space == 0 ? c->globT_off : c->globS_off);
    for (int64_t t = 0; t < nown; ++t) {
      const int64_t g = base + t;
      const int ijk[3] = {(int)(g % N0), (int)((g / N0) % N1), (int)(g / ((int64_t)N0 * N1))};
      double p[3] = {0, 0, 0};
      for (int s = 0; s < 3; ++s) if (c->perm[s] >= 0) p[c->perm[s]] = (*X[s])[ijk[s]];
      for (int a = 0; a < 3; ++a) xyz[3 * t + a] = p[a];
    }
  } else {
    const int nl = 1 << c->dim;
    const int C0 = std::max(1, c->Ncell_glob[0]), C1 = std::max(1, c->Ncell_glob[1]);
    const int act[3] = {1, c->perm[1] >= 0, c->perm[2] >= 0};
    const int64_t cell0 = (space == 0 ? c->globT_off : c->globS_off) / nl;  // first owned cell (global)
    for (int64_t t = 0; t < nown; ++t) {
      const int64_t cell = cell0 + t / nl;
      const int l = (int)(t % nl);
      const int ci[3] = {(int)(cell % C0), (int)((cell / C0) % C1), (int)(cell / ((int64_t)C0 * C1))};
      int bits[3] = {0, 0, 0}, k = 0;
      for (int s = 0; s < 3; ++s) {
        if (!act[s]) continue;
        bits[s] = (l >> k) & 1;
        ++k;
      }
      double p[3] = {0, 0, 0};
      for (int s = 0; s < 3; ++s) if (c->perm[s] >= 0) p[c->perm[s]] = (*X[s])[ci[s] + bits[s]];
      for (int a = 0; a < 3; ++a) xyz[3 * t + a] = p[a];
    }
  }
  return TV_OK;
}


int tv_set_field(void* ctx, int field, const double* host, size_t n) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !host) return TV_ERR_ARG;
  hipSetDevice(c->device);
  // local only: no communication here (a host edit on some ranks must not make
  // only those ranks enter an exchange); the ghost planes of T / T_prev are
  // refreshed collectively at the start of every tv_step / tv_solve_T
  int rc = transfer(c, field, const_cast<double*>(host), n, 0);
  if (rc == TV_OK && hipStreamSynchronize(c->stream) != hipSuccess) rc = c->fail(TV_ERR_HIP, "sync");
  return rc;
}


int tv_get_field(void* ctx, int field, double* host, size_t n) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !host) return TV_ERR_ARG;
  if (c->comm_stub)  // a stubbed share solves a decoupled block: timing only, no solution to read
    return c->fail(TV_ERR_STATE, "tv_get_field: the context runs on the measurement stub (tv_comm_init_stub)");
  hipSetDevice(c->device);
  return transfer(c, field, host, n, 1);
}


int tv_field_device_ptr(void* ctx, int field, void** dev_ptr, int64_t* comp_stride) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || field < 0 || field >= TV_NUM_FIELDS) return TV_ERR_ARG;
  if (!c->f[field].ptr) return c->fail(TV_ERR_STATE, "field not materialized");
  hipSetDevice(c->device);
  HIPC(hipStreamSynchronize(c->stream));  // the queued steps are complete when the consumer reads
  if (dev_ptr) *dev_ptr = c->f[field].ptr;
  if (comp_stride) *comp_stride = field_stride(c, c->f[field].space);
  return TV_OK;
}


int tv_set_initial_condition(void* ctx, double T0) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  hipSetDevice(c->device);
  // __set_IC_T, __set_IC_Tf, __set_IC_Tf_partial (ThermoViscoProblem.py:193-233)
  launch_fill(c->f[TV_F_T].ptr, c->nT, T0, c->stream);
  launch_fill(c->f[TV_F_T_PREV].ptr, c->nT, T0, c->stream);
  launch_fill(c->f[TV_F_TF].ptr, c->nT, T0, c->stream);
  launch_fill(c->f[TV_F_TF_PARTIAL].ptr, field_stride(c, 0) * 6, T0, c->stream);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}


// ---- time-series output (ThermoViscoProblem.py:246-276, 357-364, 614-620) ----
int tv_output_open(void* ctx, const char* dir, const int* field_ids, int n_fields) {
  return tv_output_open_named(ctx, dir, field_ids, nullptr, n_fields);
}

int tv_output_open_named(void* ctx, const char* dir, const int* field_ids, const char* const* series_names,
                         int n_fields) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !dir || !field_ids || n_fields < 1) return TV_ERR_ARG;
  if (c->out) return c->fail(TV_ERR_STATE, "output already open");
  hipSetDevice(c->device);
  // mesh of the owned nodes (storage order; a partition keeps its owned planes)
  std::vector<std::vector<double>> Xs(3);
  int phys[3];
  std::vector<double> tmp;
  for (int sx = 0; sx < 3 && !c->um; ++sx) {
    Xs[sx] = storage_coords(c, sx, tmp);
    phys[sx] = c->perm[sx];
  }
  // CG: the owned node planes; DG: the nodes of the owned cell layers; mixed
  // families: the nodes of the owned cell layers of the DG space
  if (c->n_parts > 1 && !c->um) {
    const int end = c->mixed_part == 2 ? std::min(c->plane_end + 1, c->Nnode_glob[2])
                                       : c->plane_end + (c->fam_T == TV_DG ? 1 : 0);
    Xs[2] = std::vector<double>(Xs[2].begin() + c->plane_begin, Xs[2].begin() + end);
  }
  std::string err;
  // a partitioned unstructured mesh writes its own cells over all its local
  // vertices (the ghosts' values are kept current: visco runs on every local vertex)
  const size_t ncl = (size_t)c->um_own_cells << c->dim;
  Output* o = c->um ? output_create_unstructured(
                          dir, c->dim, c->um_xyz,
                          std::vector<int64_t>(c->um_cells.begin(), c->um_cells.begin() + std::min(ncl, c->um_cells.size())),
                          err)
                    : output_create(dir, c->dim, Xs, phys, err);
  if (!o) return c->fail(TV_ERR_STATE, "output: " + err);
  static const char* names[TV_NUM_FIELDS] = {
      "T", "T_prev", "T_next", "Tf", "Tf_prev", "Tf_partial", "Tf_partial_prev", "phi", "phi_next", "xi",
      "thermal_strain", "total_strain", "deviatoric_strain", "ds_partial", "dsigma_partial", "s_tilde_partial",
      "s_tilde_partial_next", "sigma_tilde_partial", "sigma_tilde_partial_next", "s_partial", "s_partial_next",
      "sigma_partial", "sigma_partial_next", "sigma", "residual", "dx"};
  for (int k = 0; k < n_fields; ++k) {
    const int id = field_ids[k];
    if (id < 0 || id >= TV_NUM_FIELDS || !c->f[id].ptr) {
      output_destroy(o);
      return c->fail(TV_ERR_ARG, "output: field not available");
    }
    const FieldInfo& fi = c->f[id];
    const bool dg = (fi.space == 0 ? c->fam_T : c->fam_S) == TV_DG;
    const int64_t n = (c->um && c->n_parts > 1) ? c->nT
                      : c->mixed_part ? (fi.space == 0 ? c->outT_n : c->outS_n)
                                      : (fi.space == 0) ? c->ownT_n : c->ownS_n;
    const char* nm = (series_names && series_names[k] && series_names[k][0]) ? series_names[k] : names[id];
    for (const char* q = nm; *q; ++q)
      if (*q == '/' || *q == '\\') {
        output_destroy(o);
        return c->fail(TV_ERR_ARG, "output: a series name must not contain a path separator");
      }
    if (!output_add_field(o, nm, fi.bs, dg, (size_t)n * fi.bs, err)) {
      output_destroy(o);
      return c->fail(TV_ERR_STATE, "output: " + err);
    }
  }
  if (!output_start(o, c->device, err)) {
    output_destroy(o);
    return c->fail(TV_ERR_HIP, err);
  }
  c->out = o;
  c->out_fields.assign(field_ids, field_ids + n_fields);
  return TV_OK;
}

// gathers the fields in the reference's interleaved layout into a device
// staging set on the compute stream and returns; copy and file writes overlap
// the following steps (tv_output.cpp)

int tv_output_write(void* ctx, double t) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  if (!c->out) return c->fail(TV_ERR_STATE, "output not open");
  if (c->comm_stub) return c->fail(TV_ERR_STATE, "tv_output_write: the context runs on the measurement stub");
  hipSetDevice(c->device);
  int set = 0;
  double* d = output_acquire(c->out, &set);
  for (size_t k = 0; k < c->out_fields.size(); ++k) {
    const FieldInfo& fi = c->f[c->out_fields[k]];
    const bool local_all = c->um && c->n_parts > 1;  // see tv_output_open_named
    // a mixed-family slab: the dofs of its output mesh (setup_mixed_part)
    const int64_t ndof = local_all ? c->nT
                         : c->mixed_part ? (fi.space == 0 ? c->outT_n : c->outS_n)
                                         : (fi.space == 0) ? c->ownT_n : c->ownS_n;
    const int64_t off = local_all ? 0 : (fi.space == 0) ? c->ownT_off : c->ownS_off;
    const int64_t stride = field_stride(c, fi.space);
    const bool dgsp = (fi.space == 0 ? c->fam_T : c->fam_S) == TV_DG;
    const int nl = dgsp ? (1 << c->dim) : 0;
    const int64_t ncell = dgsp ? ndof / nl : 0;
    const int64_t need = ndof * fi.bs;
    const int blocks = (int)std::min<int64_t>(std::max<int64_t>(1, (need + 255) / 256), 16384);
    hipLaunchKernelGGL(k_interleave, dim3(blocks), dim3(256), 0, c->stream, 1, d + output_offset(c->out, k), fi.ptr,
                       ndof, fi.bs, stride, off, nl, ncell);
  }
  if (hipError_t e = hipGetLastError(); e != hipSuccess) {
    output_release(c->out, set);  // the set is not submitted: give it back
    return c->fail(TV_ERR_HIP, std::string("output gather: ") + hipGetErrorString(e));
  }
  std::string err;
  if (!output_submit(c->out, set, t, c->stream, err)) return c->fail(TV_ERR_STATE, "output: " + err);
  return TV_OK;
}


int tv_output_close(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  if (!c->out) return TV_OK;
  hipSetDevice(c->device);
  const std::string e = output_destroy(c->out);
  c->out = nullptr;
  c->out_fields.clear();
  if (!e.empty()) return c->fail(TV_ERR_STATE, "output: " + e);
  return TV_OK;
}


int tv_set_dirichlet(void* ctx, int enable, double value) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  if (c->O.model_mode != TV_MODEL_PAPER)
    return c->fail(TV_ERR_STATE, "Dirichlet condition: only with model_mode = TV_MODEL_PAPER (the reference's "
                                 "own path cannot run, ThermoViscoProblem.py:236-243)");
  if (enable && c->amg_on)
    return c->fail(TV_ERR_STATE, "Dirichlet condition: not with TV_PC_AMG (Jacobi or the box multigrid)");
  hipSetDevice(c->device);
  c->dir_on = enable != 0;
  c->dir_value = value;
  if (c->dir_on && c->fam_T == TV_CG && !c->dB) {
    const size_t nb = sizeof(double) * (size_t)std::max<int64_t>(1, c->nT);
    HIPC(hipMalloc(&c->dB, nb));
    HIPC(hipMalloc(&c->dtmp, nb));
    HIPC(hipMemsetAsync(c->dtmp, 0, nb, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
  }
  return TV_OK;
}


int tv_sync(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}


int tv_get_options(void* ctx, tv_options* out) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !out) return TV_ERR_ARG;
  *out = c->O;
  return TV_OK;
}


// the attributes of the reference's problem.solver (dolfinx NewtonSolver,
// ThermoViscoProblem.py:334-337): read at the next solve; the gated step end
// queues its test with the values in force then
int tv_set_newton_tolerances(void* ctx, double rtol, double atol, int max_it, int error_on_nonconvergence) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  if (!(rtol >= 0.0) || !(atol >= 0.0) || max_it < 1)
    return c->fail(TV_ERR_ARG, "Newton tolerances: rtol >= 0, atol >= 0 and max_it >= 1");
  c->O.newton_rtol = rtol;
  c->O.newton_atol = atol;
  c->O.newton_max_it = max_it;
  c->O.error_on_nonconvergence = error_on_nonconvergence ? 1 : 0;
  return TV_OK;
}


// problem.ksp.setTolerances (PETSc KSPSetTolerances on the solver's KSP,
// ThermoViscoProblem.py:339): pcg_state_init reads them at every solve
int tv_set_ksp_tolerances(void* ctx, double rtol, double atol, double dtol, int max_it) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  if (!(rtol >= 0.0) || !(atol >= 0.0) || !(dtol > 0.0) || max_it < 1)
    return c->fail(TV_ERR_ARG, "KSP tolerances: rtol >= 0, atol >= 0, dtol > 0 and max_it >= 1");
  c->O.ksp_rtol = rtol;
  c->O.ksp_atol = atol;
  c->O.ksp_dtol = dtol;
  c->O.ksp_max_it = max_it;
  return TV_OK;
}

}  // extern "C"
