// Geometric multigrid on a slab-partitioned box: the same preconditioner as
// the single-partition V-cycle (tv_mgsolve.cpp: the same global hierarchy,
// transfers, damped-Jacobi weights and coarse operators), run by P ranks.
// Replaces the reference's distributed PCGAMG (ThermoViscoProblem.py:343-346
// under mpiexec, mesh distributed at :27-28, ghosts refreshed at :351).
//
// Levels 0 .. A - 1 are DISTRIBUTED: every rank holds its slab of the level
// (storage axis 2) with one ghost plane per interface, nested across levels --
// coarse plane I belongs to the rank that owns its fine centre (2I, or the
// last fine plane of an odd cell count), so a rank's coarse slab sits inside
// its fine one, one ghost plane either side included.  Levels A .. L - 1 are
// REPLICATED: every rank holds the whole (small) level and runs the same
// coarse V-cycle on it -- the agglomeration that keeps the number of
// latency-bound exchanges per V-cycle fixed as ranks are added.  A is the
// first coarse level with at most kMgReplicateNodes nodes (or where a rank
// would own fewer than two planes).
//
// Exchanges per V-cycle (each one RCCL group of <= 2 plane sends / receives,
// or one all-reduce):
//   down, per distributed level l: ghost planes of the pre-smoothed x_l (for
//     J x_l), then -- into a distributed level -- of the residual
//     d_l = b_l - J x_l (its restriction reads the fine planes either side of
//     a coarse plane), or -- into the replicated level A -- one all-reduce of
//     the partial restrictions (each rank restricts its owned fine nodes only,
//     ghosts masked, so the sum over ranks is the full restriction);
//   up, per distributed level l >= 1: ghost planes of the post-smoothed x_l
//     (the prolongation into level l - 1 reads coarse planes either side).
// The prolongation runs on the fine ghost planes too (its inputs are all
// local), so level 0's post-smoothing J x needs no exchange of its own.
#include "tv_ctx.h"

namespace tv {

constexpr int64_t kMgReplicateNodes = 300000;  // coarse levels this small are replicated on every rank

namespace {

// global plane -> owning part along storage axis 2, per level
std::vector<int> owners_level0(int N2, int P) {
  std::vector<int> own((size_t)N2, 0);
  for (int p = 0; p < P; ++p) {
    int b0, b1;
    part_planes(N2, P, p, &b0, &b1);
    for (int k = b0; k < b1; ++k) own[(size_t)k] = p;
  }
  return own;
}

// [lo, hi) of part p in an owner array (contiguous by construction); lo = hi = 0 if empty
void owned_range(const std::vector<int>& own, int p, int* lo, int* hi) {
  *lo = *hi = 0;
  bool found = false;
  for (size_t k = 0; k < own.size(); ++k)
    if (own[k] == p) {
      if (!found) *lo = (int)k;
      found = true;
      *hi = (int)k + 1;
    }
}

// level description of one rank
struct LevelRef {
  const CgGrid* g;
  const double* T;
  double *b, *x, *w;
  const double* dinv;
  double omega;
  int64_t off, n_own;  // first owned local node, owned node count
  int64_t woff, n_win;  // the write window (= owned, but on a deep-ghost fine slab)
};

LevelRef level_ref(Ctx* c, size_t l, const double* T0) {
  LevelRef r{};
  if (l == 0) {
    r.g = &c->cg;
    r.T = T0;
    r.b = c->r;
    r.x = c->mgx;
    r.w = c->w;
    r.dinv = c->dinv;
    r.omega = c->mg_omega0;
  } else {
    MgLevel& L = c->mg[l - 1];
    r.g = &L.g;
    r.T = L.T;
    r.b = L.b;
    r.x = L.x;
    r.w = L.w;
    r.dinv = L.dinv;
    r.omega = L.omega;
  }
  const int64_t plane = (int64_t)r.g->n0 * r.g->n1;
  r.off = plane * r.g->k_begin;
  r.n_own = plane * (r.g->k_end - r.g->k_begin);
  r.woff = plane * r.g->w_begin;
  r.n_win = plane * (r.g->w_end - r.g->w_begin);
  return r;
}

}  // namespace

int mg_setup_dist(Ctx* c) {
  if (c->fam_T != TV_CG) return c->fail(TV_ERR_ARG, "partitioned GMG: CG1 temperature space");
  const int P = c->n_parts, p = c->part;
  // AUTO = GLOBAL: block Jacobi needs ~2.4x the Krylov iterations at C4's cell
  // sizes (5 -> 10-12 per solve for 2-8 slabs, tools/mg_coupling_model.py),
  // more than its saved exchanges are worth
  const bool local = c->O.mg_coupling == TV_MG_COUPLING_LOCAL;
  c->mg_local = local;
  std::vector<double> tmp, Xf[3];
  for (int s = 0; s < 3; ++s) Xf[s] = storage_coords(c, s, tmp);
  const double da = c->P.dt * c->P.alpha;
  HIPC(hipMalloc(&c->mgx, sizeof(double) * (size_t)std::max<int64_t>(1, c->nT)));
  HIPC(hipMemsetAsync(c->mgx, 0, sizeof(double) * (size_t)std::max<int64_t>(1, c->nT), c->stream));
  c->mg_omega0 = mg_omega(mg_gershgorin(Xf, da));
  // the global hierarchy (the single-partition rule) and the plane owners of every level
  const int max_levels = c->O.mg_levels > 0 ? c->O.mg_levels : 8;
  const bool automatic = c->O.mg_levels <= 0;
  struct PlanLevel {
    std::vector<double> X[3];
    std::vector<char> is_c[3];  // (l >= 1) fine nodes of level l - 1 kept on level l
    int coarse[3] = {0, 0, 0};
    std::vector<int> owner;     // owning part of each global plane (axis 2)
  };
  std::vector<PlanLevel> plan(1);
  for (int s = 0; s < 3; ++s) plan[0].X[s] = Xf[s];
  plan[0].owner = owners_level0((int)Xf[2].size(), P);
  for (int lev = 1; lev < max_levels; ++lev) {
    PlanLevel nl;
    if (!mg_next_level(plan.back().X, da, automatic, nl.X, nl.is_c, nl.coarse)) break;
    const PlanLevel& fl = plan.back();
    for (size_t k = 0; k < fl.X[2].size(); ++k)
      if (nl.is_c[2][k]) nl.owner.push_back(fl.owner[k]);  // a coarse plane belongs to its fine centre's owner
    plan.push_back(std::move(nl));
  }
  // LOCAL coupling with automatic depth: each partition runs its own slab
  // hierarchy, which needs >= 2 planes per level on every partition -- end the
  // hierarchy at the last level where that holds (an explicit mg_levels that
  // goes deeper is refused below)
  if (local && automatic) {
    for (size_t l = 1; l < plan.size(); ++l) {
      int min_own = 1 << 30;
      for (int q = 0; q < P; ++q) {
        int lo, hi;
        owned_range(plan[l].owner, q, &lo, &hi);
        min_own = std::min(min_own, hi - lo);
      }
      if (min_own < 2) {
        plan.resize(l);
        break;
      }
    }
  }
  const int L = (int)plan.size();
  // the transfers of a partitioned level are the row kernels with table-driven
  // y / z maps (k_mg_restrict_pairs, k_mg_prolong_pairs): x must coarsen
  for (int l = 1; l < L; ++l)
    if (!plan[l].coarse[0] || plan[l - 1].X[0].size() < 3)
      return c->fail(TV_ERR_ARG, "partitioned GMG: every level must coarsen along x (>= 2 cells)");
  // distributed levels: while the level is large and every part keeps >= 2 planes
  int A = L;
  for (int l = 1; l < L; ++l) {
    const int64_t nodes = (int64_t)plan[l].X[0].size() * plan[l].X[1].size() * plan[l].X[2].size();
    int min_own = 1 << 30;
    for (int q = 0; q < P; ++q) {
      int lo, hi;
      owned_range(plan[l].owner, q, &lo, &hi);
      min_own = std::min(min_own, hi - lo);
    }
    const int64_t rep = c->O.mg_replicate_nodes > 0 ? c->O.mg_replicate_nodes : kMgReplicateNodes;
    if (min_own < 2 && local)  // a slab hierarchy needs >= 2 planes per level on every partition
      return c->fail(TV_ERR_ARG, "partitioned GMG (local coupling): a level leaves a partition with < 2 planes; "
                                 "fewer levels (mg_levels) or fewer partitions");
    if (!local && (nodes <= rep || min_own < 2)) {
      A = l;
      break;
    }
  }
  c->mg_A = A;
  // local window of each level: [first2, first2 + n2) global planes of axis 2
  std::vector<int> first2(L), n2loc(L), own_lo(L), own_hi(L);
  const int G0 = c->ghost_depth;  // level 0: kDeepGhosts planes per interface (deep ghosts), else 1
  if (G0 > 1 && local) return c->fail(TV_ERR_ARG, "partitioned GMG: deep ghosts with LOCAL coupling (internal)");
  // the single-reduction (Chronopoulos-Gear) form on a deep-ghost slab (pcg_variant
  // AUTO): its matvec u = A z right after the V-cycle needs z one plane beyond
  // the owned ones, so level 0's post-smoothing reads x two planes out and the
  // prolongation into them reads level 1 two ghost planes deep
  c->mg_cgs = G0 > 1 && c->O.pcg_variant == TV_PCG_AUTO;
  auto gdep = [&](int l) { return l == 0 ? G0 : (l == 1 && c->mg_cgs) ? 2 : 1; };  // ghost planes of level l
  // fine planes the prolongation into level l fills: within `need` planes of
  // the owned ones (every local plane where the level has one ghost plane)
  auto need = [&](int l) { return (l == 0 && c->mg_cgs) ? 2 : 1; };
  for (int l = 0; l < L; ++l) {
    owned_range(plan[l].owner, p, &own_lo[l], &own_hi[l]);
    if (l < A) {
      const int gd = gdep(l);
      const int glo = p > 0 ? gd : 0, ghi = p < P - 1 ? gd : 0;
      first2[l] = own_lo[l] - glo;
      n2loc[l] = own_hi[l] - own_lo[l] + glo + ghi;
    } else {
      first2[l] = 0;
      n2loc[l] = (int)plan[l].X[2].size();
    }
  }
  if (first2[0] != c->plane_begin - c->cg.g_lo || n2loc[0] != c->cg.n2)
    return c->fail(TV_ERR_ARG, "partitioned GMG: level-0 window differs from the partition (internal)");
  for (int l = 1; l < L; ++l) {
    c->mg.emplace_back();
    MgLevel& Lv = c->mg.back();
    const PlanLevel& pl = plan[l];
    for (int s = 0; s < 3; ++s) Lv.X[s] = pl.X[s];
    Lv.dist = l < A;
    Lv.first2 = first2[l];
    if (Lv.dist) {
      const int glo = p > 0 ? gdep(l) : 0, ghi = p < P - 1 ? gdep(l) : 0;
      if (int e = build_cg_grid(c, 3, Lv.X, first2[l], n2loc[l], glo, ghi, p == 0, p == P - 1, Lv.g, Lv.coef,
                                &Lv.bnodes, Lv.ffbuf))
        return e;
    } else {
      if (int e = build_cg_grid(c, 3, Lv.X, 0, n2loc[l], 0, 0, true, true, Lv.g, Lv.coef, &Lv.bnodes, Lv.ffbuf))
        return e;
    }
    if (int e = mg_level_vectors(c, Lv)) return e;
    Lv.omega = mg_omega(mg_gershgorin(Lv.X, da));  // over the global level: the same on every rank
    // the coarse planes whose T this rank injects: its own ones
    Lv.inj0 = own_lo[l] - first2[l];
    Lv.inj1 = own_hi[l] - first2[l];
    // transfer tables (level l - 1 -> l), axes 0 and 1 whole, axis 2 over the local windows
    MgXfer& x = Lv.xf;
    const PlanLevel& fp = plan[l - 1];
    int reach_lo = 1 << 30, reach_hi = 0;
    for (int s = 0; s < 3; ++s) {
      std::vector<int> pi, ri;
      std::vector<double> pw, rw;
      mg_axis_tables(fp.X[s], pl.is_c[s], pi, pw, ri, rw);
      int nf = (int)fp.X[s].size(), nc = (int)pl.X[s].size();
      if (s == 2) {
        const int f0 = first2[l - 1], c0 = first2[l];
        if (l == A) {  // the coarse planes this rank's owned fine planes restrict to
          for (int I = 0; I < (int)pl.X[2].size(); ++I)
            for (int q = 0; q < 3; ++q) {
              const int f = ri[3 * (size_t)I + q];
              if (rw[3 * (size_t)I + q] != 0.0 && f >= own_lo[l - 1] && f < own_hi[l - 1]) {
                reach_lo = std::min(reach_lo, I);
                reach_hi = std::max(reach_hi, I + 1);
              }
            }
        }
        nf = n2loc[l - 1];
        nc = n2loc[l];
        std::vector<int> piL(2 * (size_t)nf), riL(3 * (size_t)nc);
        std::vector<double> pwL(2 * (size_t)nf), rwL(3 * (size_t)nc);
        // LOCAL coupling (block Jacobi): a fine plane interpolates only from the
        // coarse planes this partition owns and a coarse plane restricts only
        // from owned fine planes (R = P^T of the slab); excluded entries keep
        // weight 0 and point at an owned plane (finite data)
        const int cown0 = own_lo[l] - c0, cown1 = own_hi[l] - c0;
        const int fown0 = own_lo[l - 1] - f0, fown1 = own_hi[l - 1] - f0;
        // deep ghosts: the prolongation fills the fine planes within need(l - 1)
        // of the owned ones -- all the post-smoothing J x reads; the outer
        // ghost planes keep x0 and take no weight
        const int skip = (l - 1 < A) ? std::max(0, gdep(l - 1) - need(l - 1)) : 0;
        const int fin0 = p > 0 ? skip : 0, fin1 = p < P - 1 ? nf - skip : nf;
        for (int lf = 0; lf < nf; ++lf)
          for (int e = 0; e < 2; ++e) {
            const int cg = pi[2 * (size_t)(f0 + lf) + e] - c0;  // coarse local
            if (!local && (lf < fin0 || lf >= fin1)) {
              piL[2 * (size_t)lf + e] = std::min(std::max(cg, 0), nc - 1);
              pwL[2 * (size_t)lf + e] = 0.0;
              continue;
            }
            const bool ok = local ? (cg >= cown0 && cg < cown1 && lf >= fown0 && lf < fown1) : (cg >= 0 && cg < nc);
            if (local && !ok) {
              piL[2 * (size_t)lf + e] = std::min(std::max(cg, cown0), cown1 - 1);
              pwL[2 * (size_t)lf + e] = 0.0;
              continue;
            }
            // every fine local plane interpolates from coarse local planes (nesting)
            if (!ok && pw[2 * (size_t)(f0 + lf) + e] != 0.0)
              return c->fail(TV_ERR_ARG, "partitioned GMG: prolongation leaves the local window (internal)");
            piL[2 * (size_t)lf + e] = ok ? cg : 0;
            pwL[2 * (size_t)lf + e] = ok ? pw[2 * (size_t)(f0 + lf) + e] : 0.0;
          }
        for (int lc = 0; lc < nc; ++lc)
          for (int q = 0; q < 3; ++q) {
            const int fgl = ri[3 * (size_t)(c0 + lc) + q] - f0;  // fine local
            const bool ok = local ? (fgl >= fown0 && fgl < fown1 && lc >= cown0 && lc < cown1) : (fgl >= 0 && fgl < nf);
            if (local && !ok) {
              riL[3 * (size_t)lc + q] = std::min(std::max(fgl, fown0), fown1 - 1);
              rwL[3 * (size_t)lc + q] = 0.0;
              continue;
            }
            // outside the fine window (a coarse ghost plane's far side, or a coarse
            // plane of the replicated level away from this slab): weight 0, and the
            // restriction never writes those planes from this rank's data
            riL[3 * (size_t)lc + q] = ok ? fgl : std::min(std::max(fgl, 0), nf - 1);
            rwL[3 * (size_t)lc + q] = ok ? rw[3 * (size_t)(c0 + lc) + q] : 0.0;
          }
        pi.swap(piL);
        pw.swap(pwL);
        ri.swap(riL);
        rw.swap(rwL);
      }
      if (int e = mg_upload(c, Lv, pi, &x.pi[s])) return e;
      if (int e = mg_upload(c, Lv, pw, &x.pw[s])) return e;
      if (int e = mg_upload(c, Lv, ri, &x.ri[s])) return e;
      if (int e = mg_upload(c, Lv, rw, &x.rw[s])) return e;
      x.fn[s] = nf;
      x.cn[s] = nc;
      x.coarse[s] = pl.coarse[s];
    }
    // prolongation into every local fine plane (ghost planes included; LOCAL:
    // the owned ones, the ghost planes of a slab's V-cycle stay zero)
    x.f_kb = local ? own_lo[l - 1] - first2[l - 1] : 0;
    x.f_ke = local ? own_hi[l - 1] - first2[l - 1] : x.fn[2];
    if (!local && l - 1 < A) {  // deep ghosts: within need(l - 1) planes of the owned fine planes
      const int skip = std::max(0, gdep(l - 1) - need(l - 1));
      x.f_kb = p > 0 ? skip : 0;
      x.f_ke = p < P - 1 ? x.fn[2] - skip : x.fn[2];
    }
    if (Lv.dist) {  // restriction: the owned coarse planes
      x.c_kb = Lv.g.k_begin;
      x.c_ke = Lv.g.k_end;
      x.aligned = 0;
    } else if (l == A) {
      // restriction into the replicated level: every coarse plane -- the ones
      // this rank's owned fine planes reach get its masked partial sums (which
      // add up over the ranks), the others exact zeros (weight-0 entries), so
      // the level vector needs no zero fill before it (a 4.7 us launch per
      // V-cycle at the C4 / 8 share)
      (void)reach_lo;
      (void)reach_hi;
      x.c_kb = 0;
      x.c_ke = x.cn[2];
      x.aligned = 0;
    } else {
      x.c_kb = 0;
      x.c_ke = x.cn[2];
      x.aligned = 1;
    }
  }
  // restriction mask of the last distributed level (ghost planes out)
  if (A < L) {
    const LevelRef r = level_ref(c, (size_t)(A - 1), nullptr);
    const int64_t nloc = (int64_t)r.g->n0 * r.g->n1 * r.g->n2;
    double** m = (A - 1 == 0) ? &c->mg_mask0 : &c->mg[A - 2].mask;
    HIPC(hipMalloc(m, sizeof(double) * (size_t)std::max<int64_t>(1, nloc)));
    launch_mg_ownmask(nloc, r.off, r.off + r.n_own, nullptr, *m, c->stream);
    HIPC(hipGetLastError());
  }
  if (c->mg_cgs) {  // s = A p of the single-reduction form
    HIPC(hipMalloc(&c->mg_s, sizeof(double) * (size_t)std::max<int64_t>(1, c->nT)));
    HIPC(hipMemsetAsync(c->mg_s, 0, sizeof(double) * (size_t)std::max<int64_t>(1, c->nT), c->stream));
  }
  c->mg_on = true;
  return TV_OK;
}

// per Newton iteration: T of every coarse level (distributed levels: injected
// on the owned planes, then the ghost planes exchanged; the first replicated
// level: each rank injects its own planes into a zeroed vector, summed over
// the ranks; below it, injected locally) and the Jacobi diagonals
int mg_prepare_dist(Ctx* c, const double* T) {
  if (c->mg_dg) return mg_prepare(c, T);  // a DG1 slab: level 1 onwards replicated (mg_setup)
  const double* Tf = T;
  for (size_t l = 1; l <= c->mg.size(); ++l) {
    MgLevel& L = c->mg[l - 1];
    if (L.dist) {
      launch_mg_inject_range(L.xf, Tf, L.T, L.inj0, L.inj1, c->stream);
      if (int e = halo_grid(c, L.g, L.T)) return e;
    } else if ((int)l == c->mg_A) {
      HIPC(hipMemsetAsync(L.T, 0, sizeof(double) * (size_t)L.n, c->stream));
      launch_mg_inject_range(L.xf, Tf, L.T, L.inj0, L.inj1, c->stream);
      if (int e = allreduce_vec(c, L.T, L.n)) return e;
    } else {
      launch_mg_inject(L.xf, Tf, L.T, c->stream);
    }
    launch_cg_diag(L.g, L.T, L.dinv, 1, c->stream, L.dinv_interior);
    L.dinv_interior = true;
    Tf = L.T;
  }
  HIPC(hipGetLastError());
  return TV_OK;
}

// V-cycle; on entry x_0 = omega0 D^-1 r on the owned nodes of level 0 (the
// KSPCG update); on exit z (owned) = the V-cycle applied to r and the (z.z,
// z.r) records reduced into c->sums by the tail (kind 0: the all-reduce and
// the KSPCG logic follow).  Returns a status.
int mg_apply0_dist(Ctx* c, const double* T, const RedTail* tail) {
  if (c->amg_on || c->mg_dg) {  // the agglomerated algebraic cycle (tv_amg.cpp); a DG1 slab (tv_mgsolve.cpp)
    const int r = c->amg_on ? amg_apply0(c, tail) : mg_apply0(c, T, tail);
    return r < 0 ? -r : TV_OK;
  }
  hipStream_t s = c->stream;
  const size_t L = c->mg.size() + 1;  // levels incl. 0
  const size_t A = (size_t)c->mg_A;
  const double* dmask = c->dir_on ? c->dinv : nullptr;  // Dirichlet: the free subspace (level 0)
  const size_t ldown = std::min(A, L);  // distributed levels
  // the V-cycle's ghost exchanges (LOCAL coupling: none -- the slab's own cycle,
  // whose ghost planes hold zeros)
  auto vhalo = [&](const CgGrid& g, double* v) -> int { return c->mg_local ? TV_OK : halo_grid(c, g, v); };
  // deep ghosts: level 0's x0 (the KSPCG update) and residual d0 are computed
  // on the write window -- every ghost plane but the outermost -- from
  // vectors that are valid there, so neither needs an exchange (two exchange
  // points fewer per V-cycle); the closing group refreshes z's kDeepGhosts planes
  const bool deep = c->ghost_depth > 1;
  // ---- down: distributed levels 0 .. A - 1
  for (size_t l = 0; l < ldown; ++l) {
    const LevelRef r = level_ref(c, l, T);
    if (!(deep && l == 0))
      if (int e = vhalo(*r.g, r.x)) return e;  // ghosts of the pre-smoothed x_l
    if (l + 1 == L) break;                           // the coarsest level, distributed: x_l is its solve
    launch_cg_japply_partial(*r.g, r.T, r.x, r.w, c->st, s);
    FaceAdd fa = cg_face_add(*r.g, r.woff);
    MgLevel& C = c->mg[l];
    if (l + 1 < A) {  // into a distributed level: exchange the residual, restrict on the owned coarse planes
      launch_mg_resid(r.n_win, c->st, r.b + r.woff, r.w + r.woff, &fa, l == 0 && dmask ? dmask + r.woff : nullptr, s);
      if (!(deep && l == 0))
        if (int e = vhalo(*r.g, r.w)) return e;
      launch_mg_restrict(C.xf, c->st, r.w, nullptr, nullptr, nullptr, C.b, C.dinv, C.omega, C.x, s);
    } else {  // into the replicated level A: masked partial restriction, summed over the ranks
      const double* mask = (l == 0) ? c->mg_mask0 : c->mg[l - 1].mask;
      const FaceAdd fa0 = cg_face_add(*r.g, 0);
      launch_mg_restrict(C.xf, c->st, r.b, r.w, &fa0, mask, C.b, nullptr, 0.0, nullptr, s);
      if (int e = allreduce_vec(c, C.b, C.n)) return e;
      launch_mg_jacobi(C.n, c->st, C.b, nullptr, nullptr, C.dinv, C.omega, C.x, 0, s);  // pre-smoothing from 0
      mg_level(c, A);  // the replicated V-cycle below (single-partition code; post-smooths level A)
    }
  }
  // ---- up: prolongation into the distributed levels, post-smoothing, ghosts
  for (size_t l = std::min(A, L - 1); l-- > 0;) {
    const LevelRef r = level_ref(c, l, T);
    MgLevel& C = c->mg[l];
    // every local fine plane, ghost planes included (their inputs are local)
    launch_mg_prolong(C.xf, c->st, r.x, C.x, l == 0 ? dmask : nullptr, s);
    // loopback transport test only (tv_comm_init_loopback: the neighbours are
    // this slab's periodic images): the ghost planes prolongated from the
    // replicated GLOBAL level are not the images of the owned ones, so they are
    // refreshed from them -- on a real partition the exchange would deliver
    // exactly what the prolongation computed there (a no-op, never issued)
    if (c->comm_self && l + 1 == A && A < L)
      if (int e = vhalo(*r.g, r.x)) return e;
    // level 0: J x, the post-smoothing and the (z.z, z.r) records in the march
    // epilogue (+ the side-face pass with the reduction tail), as on one partition
    if (l == 0 && launch_cg_japply_post(*r.g, r.T, r.x, r.b, r.dinv, r.omega, c->z, c->st, c->partials, tail, s) >= 0)
      return TV_OK;
    launch_cg_japply_partial(*r.g, r.T, r.x, r.w, c->st, s);
    const FaceAdd fa = cg_face_add(*r.g, r.off);
    if (l > 0) {
      launch_mg_jacobi(r.n_own, c->st, r.b + r.off, r.w + r.off, &fa, r.dinv + r.off, r.omega, r.x + r.off, 1, s);
      if (int e = vhalo(*r.g, r.x)) return e;
    } else {
      launch_mg_post(r.n_own, c->st, r.x + r.off, r.b + r.off, r.w + r.off, &fa, r.dinv + r.off, r.omega,
                     c->z + r.off, c->partials, tail, s);
      return TV_OK;
    }
  }
  // no coarse level: the two smoothing steps of level 0 only
  const LevelRef r = level_ref(c, 0, T);
  launch_cg_japply_partial(*r.g, r.T, r.x, r.w, c->st, s);
  const FaceAdd fa = cg_face_add(*r.g, r.off);
  launch_mg_post(r.n_own, c->st, r.x + r.off, r.b + r.off, r.w + r.off, &fa, r.dinv + r.off, r.omega,
                 c->z + r.off, c->partials, tail, s);
  return TV_OK;
}

namespace {

// fold: the box march path -- the scalar logic after each all-reduce runs
// lagged inside the next launch (lagged_state) instead of as a one-thread
// launch: the beta / convergence logic of the previous iteration's closing
// group inside this iteration's fused matvec (lag3), the alpha logic inside
// the update.  Every rank forms the same state from the same all-reduced sums.
}  // namespace

// the level-0 nodes a partition's pointwise V-cycle kernels cover: the owned
// ones, or on a deep-ghost slab the write window (every ghost plane but the
// outermost: x0 = omega D^-1 r is needed there, so J x0 is right one plane out)
void fine_window(const Ctx* c, int64_t* off, int64_t* n) {
  if (c->um || c->fam_T != TV_CG) {
    *off = c->ownT_off;
    *n = c->ownT_n;
    return;
  }
  const int64_t plane = (int64_t)c->cg.n0 * c->cg.n1;
  *off = plane * c->cg.w_begin;
  *n = plane * (c->cg.w_end - c->cg.w_begin);
}

namespace {

int mg_iteration_dist(Ctx* c, const double* T, int it, bool fold, bool lag3) {
  int64_t off, n;
  fine_window(c, &off, &n);
  const int slot = c->ts_next + it;
  uint64_t* ts = (c->ktime && (it % c->kstride) == 0 && slot < kTsCap) ? c->d_ts + 4 * slot : nullptr;
  RedTail t1{c->counters, c->partials, c->sums, c->st, 0, ts};
  if (lag3) {
    t1.lag = c->sums;
    t1.lag_kind = 3;
  }
  int np = 0;
  bool lag2 = false;
  if (!op_japply_fused(c, T, &np, &t1, it)) {  // p <- z + b p ; w <- J p ; p.w
    if (lag3) return c->fail(TV_ERR_STATE, "lagged PCG logic without the fused march");
    if (int e = reduce_logic(c, np, 1, 2, 1)) return e;
  } else {
    if (int e = allreduce(c, c->sums, 1)) return e;
    if (fold) lag2 = true;
    else launch_logic(c->st, c->sums, 2, c->stream);  // alpha
  }
  if (c->dggface) {  // a DG1 slab: the cell-block update (the alpha logic ran above: no fold on DG)
    launch_dg_bupdate(c->dg, c->st, c->pA, c->pB, c->w, c->dggface, c->mg_omega0, c->r, c->f[TV_F_DX].ptr, c->mgx, it,
                      0, c->stream);
  } else {
    const FaceAdd fa = c->um ? FaceAdd{} : cg_face_add(c->cg, off);  // unstructured: w is complete
    launch_mg_update(n, c->st, c->pA + off, c->pB + off, c->w + off, &fa, c->dinv + off, c->mg_omega0, c->r + off,
                     c->f[TV_F_DX].ptr + off, c->mgx + off, it, 0, c->stream, lag2 ? c->sums : nullptr,
                     lag2 ? c->counters + kUpdateCounter : nullptr);
  }
  RedTail t2{c->counters + kTailCounters, c->partials, c->sums, c->st, 0, nullptr};
  return mg_apply0_dist(c, T, &t2);
}

}  // namespace

// The single-reduction (Chronopoulos-Gear) form of the GMG-preconditioned CG
// on deep-ghost slabs (c->mg_cgs): per iteration the update (k_mg_update_cgs:
// the scalars from the lagged all-reduced sums, s, p, dx, r, x0), the V-cycle
// (z = M r with z.z, z.r), the matvec u = A z (with z.u) and ONE RCCL group --
// the all-reduce of the three sums and the ghost planes of u.  Exchange points
// per iteration: that group and the V-cycle's level-1 ghosts (pre / post) and
// the replicated level's all-reduce: 4, against 7 for KSPCG with one ghost
// plane.  Same iterates as KSPCG in exact arithmetic
// (PETSc KSPCG's tests on ||z|| and (z, r), iteration counts alike).
static int pcg_solve_mg_dist_cgs(Ctx* c, const double* T, int* its, int* reason, bool post) {
  const int64_t off = c->ownT_off, n = c->ownT_n;
  int64_t woff, nwin;
  fine_window(c, &woff, &nwin);
  const PcgState h = pcg_state_init(c);
  c->h_st[2] = h;
  launch_set_state(c->st, h, c->stream, c->solve_gate);
  if (int e = mg_prepare_dist(c, T)) return e;
  if (c->dir_on)
    if (int e = halo(c, c->dinv)) return e;
  if (c->mg_mask0) launch_mg_ownmask(c->nT, off, off + n, c->dir_on ? c->dinv : nullptr, c->mg_mask0, c->stream);
  launch_mg_update(nwin, c->st, c->pA + woff, c->pB + woff, c->w + woff, nullptr, c->dinv + woff, c->mg_omega0,
                   c->r + woff, c->f[TV_F_DX].ptr + woff, c->mgx + woff, 0, 1, c->stream);  // x0 <- omega dinv r
  double* u = c->w;  // A z, completed on the ghost planes by the closing group
  int pending = 0;   // logic kind of the last closing group still to run (inside the next update)
  // V-cycle (z, z.z, z.r -> sums[0..1]), u = A z (z.u -> sums[2]), the closing group
  auto half = [&](int it) -> int {
    RedTail tz{c->counters + kTailCounters, c->partials, c->sums, c->st, 0, nullptr};
    if (int e = mg_apply0_dist(c, T, &tz)) return e;
    const int slot = c->ts_next + it;
    uint64_t* ts = (it >= 0 && c->ktime && (it % c->kstride) == 0 && slot < kTsCap) ? c->d_ts + 4 * slot : nullptr;
    RedTail tu{c->counters, c->partials, c->sums + 2, c->st, 0, ts};
    if (!launch_cg_japply_tail(c->cg, T, c->z, u, c->st, c->partials, &tu, c->stream))
      return c->fail(TV_ERR_STATE, "single-reduction GMG needs the marching matvec (internal)");
    if (int e = allreduce_halo(c, c->sums, 3, u)) return e;
    pending = it < 0 ? 7 : 6;
    return TV_OK;
  };
  if (int e = half(-1)) return e;  // iteration 0's z, u and sums
  if (c->ktime && c->ts_next + c->O.ksp_max_it + 8 > kTsCap)
    if (int e = ts_flush(c)) return e;
  int launched = 0;
  auto enqueue = [&](int nb) -> int {
    for (int b = 0; b < nb; ++b) {
      const int it = launched + b;
      launch_mg_update_cgs(nwin, c->st, u + woff, c->mg_s + woff, c->z + woff, c->pA + woff, c->f[TV_F_DX].ptr + woff,
                           c->r + woff, c->dinv + woff, c->mg_omega0, c->mgx + woff, it == 0,
                           pending ? c->sums : nullptr, pending, c->counters + kUpdateCounter, c->stream);
      pending = 0;
      if (int e = half(it)) return e;
    }
    launched += nb;
    if (pending) {  // the host polls the state: the last group's logic as a launch of its own
      launch_logic(c->st, c->sums, pending, c->stream);
      pending = 0;
    }
    HIPC(hipGetLastError());
    if (int e = publish(c, &c->h_st[0], c->st, sizeof(PcgState))) return e;
    HIPC(hipEventRecord(c->evp[0], c->stream));
    if (post) {  // dx is complete (the updates apply it); the group zeroes it after a 0-iteration solve
      double* nrm = c->sums + 6;
      launch_post_group(n, c->st, nullptr, nullptr, c->f[TV_F_DX].ptr + off, c->f[TV_F_T].ptr + off, c->partials, nrm,
                        c->stream);
      if (int e = allreduce(c, nrm, 1)) return e;
      if (int e = queue_newton_norm(c, nrm)) return e;
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
  if (!post && *its == 0) launch_fill(c->f[TV_F_DX].ptr + off, n, 0.0, c->stream);
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

int pcg_solve_mg_dist(Ctx* c, const double* T, int* its, int* reason, bool post) {
  if (c->mg_cgs) return pcg_solve_mg_dist_cgs(c, T, its, reason, post);
  const int64_t off = c->ownT_off, n = c->ownT_n;
  int64_t woff, nwin;
  fine_window(c, &woff, &nwin);
  const PcgState h = pcg_state_init(c);
  c->h_st[2] = h;
  launch_set_state(c->st, h, c->stream, c->solve_gate);
  if (c->amg_on) {  // the algebraic hierarchy is T-independent; level 0's weight at the first solve
    if (int e = mg_dg_weight(c, T)) return e;
  } else if (int e = mg_prepare_dist(c, T)) {
    return e;
  }
  if (c->dir_on)  // the prolongation masks level 0's ghost planes with dinv too
    if (int e = halo(c, c->dinv)) return e;
  if (c->mg_mask0)  // level 0's restriction mask: owned nodes, Dirichlet rows out
    launch_mg_ownmask(c->nT, off, off + n, c->dir_on ? c->dinv : nullptr, c->mg_mask0, c->stream);
  if (c->dggface) {  // a DG1 slab: x0 <- omega B^-1 r over the owned cells
    if (int e = mg_dg_weight(c, T)) return e;
    launch_dg_bupdate(c->dg, c->st, c->pA, c->pB, c->w, c->dggface, c->mg_omega0, c->r, c->f[TV_F_DX].ptr, c->mgx, 0, 1,
                      c->stream);
  } else {
    launch_mg_update(nwin, c->st, c->pA + woff, c->pB + woff, c->w + woff, nullptr, c->dinv + woff, c->mg_omega0,
                     c->r + woff, c->f[TV_F_DX].ptr + woff, c->mgx + woff, 0, 1, c->stream);  // x0 <- omega dinv r
  }
  // the three collectives of an iteration close it: the (z.z, z.r) all-reduce
  // + KSPCG logic, and the ghost planes of z for the next fused matvec
  // the lagged logic needs the box march's fused matvec (not the unstructured
  // or DG kernels)
  const bool fold = !c->um && c->fam_T == TV_CG && cg_cgs_supported(c->cg);
  bool lag3 = false;  // the last closing group's logic is still to run (inside the next fused matvec)
  auto close = [&](int kind, bool defer) -> int {  // one RCCL group: the sums and the ghosts of z
    if (int e = allreduce_halo(c, c->sums, 2, c->z)) return e;
    if (defer) {
      lag3 = true;
    } else {
      launch_logic(c->st, c->sums, kind, c->stream);
      lag3 = false;
    }
    return TV_OK;
  };
  {
    RedTail t0{c->counters + kTailCounters, c->partials, c->sums, c->st, 0, nullptr};
    if (int e = mg_apply0_dist(c, T, &t0)) return e;
    if (int e = close(1, false)) return e;  // dp, beta (KSPCG init)
  }
  if (c->ktime && c->ts_next + c->O.ksp_max_it + 8 > kTsCap)
    if (int e = ts_flush(c)) return e;
  // queued as in pcg_solve_mg: the previous solve's count behind the init, then
  // one iteration per poll.  Every rank takes the same decisions: the polled
  // state is formed from all-reduced sums, identical on every rank.
  int launched = 0;
  auto enqueue = [&](int nb) -> int {
    for (int b = 0; b < nb; ++b) {
      if (int e = mg_iteration_dist(c, T, launched + b, fold, lag3)) return e;
      // z.z, z.r -> beta, convergence: lagged into the next iteration's fused
      // matvec, except after the batch's last iteration (the host polls the state)
      if (int e = close(3, fold && b + 1 < nb)) return e;
    }
    launched += nb;
    HIPC(hipGetLastError());
    if (int e = publish(c, &c->h_st[0], c->st, sizeof(PcgState))) return e;
    HIPC(hipEventRecord(c->evp[0], c->stream));
    if (post) {  // the Newton iteration's next work, gated on the (all-reduced, rank-identical) state
      double* nrm = c->sums + 6;  // not c->sums: the lagged logic reads those across the batch boundary
      launch_post_group(n, c->st, c->pA + off, c->pB + off, c->f[TV_F_DX].ptr + off, c->f[TV_F_T].ptr + off,
                        c->partials, nrm, c->stream);
      if (int e = allreduce(c, nrm, 1)) return e;  // collective on every rank, run or gated off
      if (int e = queue_newton_norm(c, nrm)) return e;
    }
    return TV_OK;
  };
  const int hk = std::min(c->newton_k, 15);  // every rank polls the same all-reduced state: same decisions
  if (int e = enqueue(std::max(1, c->mg_hint[hk] > 0 ? c->mg_hint[hk] : c->pcg_hint))) return e;
  for (;;) {
    HIPC(hipEventSynchronize(c->evp[0]));
    if (c->h_st[0].done) break;
    if (launched > c->O.ksp_max_it + 2) return c->fail(TV_ERR_KSP, "PCG: iteration guard exceeded");
    if (int e = enqueue(1)) return e;
  }
  *its = c->h_st[0].it;
  *reason = c->h_st[0].reason;
  if (!post) launch_mg_dx_finish(n, c->st, c->pA + off, c->pB + off, c->f[TV_F_DX].ptr + off, *its, c->stream);
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
