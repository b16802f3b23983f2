// Communication of the partitioned (multi-GPU) path: ghost-plane exchanges
// and reductions over RCCL (production, one process per GPU over xGMI) or the
// host-staged callbacks (several partitions on one GPU, tests).  Replaces the
// reference's MPI layer: dolfinx Scatterer::scatter_forward
// (ThermoViscoProblem.py:351) and PETSc's MPI_Allreduce in VecNorm / VecDot [3P].
#include "tv_ctx.h"

namespace tv {
// --------------------------------------------------------------------------------------
// communication
// --------------------------------------------------------------------------------------
bool multi_rank(const Ctx* c) { return c->nranks > 1 && (c->comm || c->host_sendrecv || c->comm_stub); }

int require_comm(Ctx* c, const char* what) {
  if (c->n_parts > 1 && !multi_rank(c))
    return c->fail(TV_ERR_STATE, std::string(what) + ": a partition of a partitioned mesh needs its communicator "
                                 "(tv_comm_init / tv_comm_init_host) before it solves");
  return TV_OK;
}

int refresh_dirty_ghosts(Ctx* c) {
  // partitioned unstructured meshes and mixed-family slabs run the visco T pass
  // on their ghost dofs too (their sigma pass / writers read them)
  if (!((c->um && c->n_parts > 1) || c->mixed_part) || !multi_rank(c) || c->comm_stub) return TV_OK;
  // T and T_prev are exchanged every step anyway (newton); the other fields
  // only when a rank wrote them.  Every rank learns the union of the writes
  // through one all-reduce of a flag per field.
  if (!c->d_dirty) HIPC(hipMalloc(&c->d_dirty, sizeof(double) * TV_NUM_FIELDS));
  double fl[TV_NUM_FIELDS];
  for (int f = 0; f < TV_NUM_FIELDS; ++f) fl[f] = (c->ghost_dirty >> f) & 1u ? 1.0 : 0.0;
  HIPC(hipMemcpyAsync(c->d_dirty, fl, sizeof(fl), hipMemcpyHostToDevice, c->stream));
  if (int e = allreduce_vec(c, c->d_dirty, TV_NUM_FIELDS)) return e;
  HIPC(hipMemcpyAsync(fl, c->d_dirty, sizeof(fl), hipMemcpyDeviceToHost, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  c->ghost_dirty = 0;
  bool tilde = false;
  for (int f = 0; f < TV_NUM_FIELDS; ++f) {
    if (fl[f] == 0.0 || !c->f[f].ptr || f == TV_F_T || f == TV_F_T_PREV) continue;
    if (c->mixed_part && c->f[f].space != 0) continue;  // the sigma space of a mixed slab has no ghosts
    const int64_t stride = field_stride(c, c->f[f].space);  // unstructured: the same vertex set (CG1 / CG1)
    for (int k = 0; k < c->f[f].bs; ++k)
      if (int e = halo(c, c->f[f].ptr + k * stride)) return e;
    tilde = tilde || f == TV_F_S_TILDE || f == TV_F_S_TILDE_NEXT || f == TV_F_SIGMA_TILDE || f == TV_F_SIGMA_TILDE_NEXT;
  }
  if (tilde) {  // a neighbour's non-zero tilde values may now sit in this rank's ghosts
    static const int one = 1;
    HIPC(hipMemcpyAsync(c->tflag, &one, sizeof(int), hipMemcpyHostToDevice, c->stream));
  }
  return TV_OK;
}

// RCCL peer of partition q: itself on a loopback communicator (one rank, peer 0)
static inline int peer(const Ctx* c, int q) { return c->comm_self ? 0 : q; }

// measurement stub (tv_comm_init_stub): the ghosts of the solver's vectors read
// zero (each partition solves its own block: the operators stay SPD), the
// temperature ghosts keep their initial value, reductions stay local.  Both
// ghost planes in ONE small launch (two hipMemsetAsync fills cost ~5 us each:
// ~2 ms of a C4 / 8 share step went into the stand-ins for its exchanges)
__global__ __launch_bounds__(kBlock) void k_zero_ghosts(double* lo, double* hi, int64_t nlo, int64_t nhi) {
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < nlo + nhi; t += (int64_t)gridDim.x * kBlock) {
    if (t < nlo) lo[t] = 0.0;
    else hi[t - nlo] = 0.0;
  }
}

static int stub_ghosts(Ctx* c, const CgGrid& g, double* v) {
  if (v == c->f[TV_F_T].ptr || v == c->f[TV_F_T_PREV].ptr) return TV_OK;
  const int64_t plane = (int64_t)g.n0 * g.n1;
  if (!g.g_lo && !g.g_hi) return TV_OK;
  const int64_t nlo = plane * g.g_lo, nhi = plane * g.g_hi;
  const int nb = (int)std::min<int64_t>(1024, (nlo + nhi + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(k_zero_ghosts, dim3(nb), dim3(kBlock), 0, c->stream, v, v + plane * g.k_end, nlo, nhi);
  HIPC(hipGetLastError());
  return TV_OK;
}

// ghost planes of v on grid g (the fine grid or a distributed multigrid level,
// storage axis 2): g_lo / g_hi planes per interface (1, or kDeepGhosts on a
// deep-ghost fine slab) -- send the first / last g owned planes (one
// contiguous block each), receive into the ghost planes below / above
int halo_host(Ctx* c, const CgGrid& g, double* v) {
  const int64_t plane = (int64_t)g.n0 * g.n1;
  const int64_t nlo = plane * g.g_lo, nhi = plane * g.g_hi;
  double* s_lo = c->h_halo;
  double* s_hi = c->h_halo + nlo;
  double* r_lo = c->h_halo + nlo + nhi;
  double* r_hi = c->h_halo + 2 * nlo + nhi;
  if (nlo) HIPC(hipMemcpyAsync(s_lo, v + plane * g.k_begin, nlo * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  if (nhi) HIPC(hipMemcpyAsync(s_hi, v + plane * (g.k_end - g.g_hi), nhi * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  if (nlo && c->host_sendrecv(s_lo, (size_t)nlo, c->rank - 1, r_lo, (size_t)nlo, c->rank - 1, c->host_user))
    return c->fail(TV_ERR_COMM, "host sendrecv failed");
  if (nhi && c->host_sendrecv(s_hi, (size_t)nhi, c->rank + 1, r_hi, (size_t)nhi, c->rank + 1, c->host_user))
    return c->fail(TV_ERR_COMM, "host sendrecv failed");
  if (c->comm_self && g.g_lo && g.g_hi) {  // loopback, both sides: periodic images (see group_planes)
    HIPC(hipMemcpyAsync(v, r_hi, nlo * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPC(hipMemcpyAsync(v + plane * g.k_end, r_lo, nhi * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    return TV_OK;
  }
  if (c->comm_self && (g.g_lo > 1 || g.g_hi > 1)) {
    // loopback, one side: the received planes land mirrored (see group_planes)
    for (int j = 0; j < g.g_lo; ++j)  // ghost plane k_begin - 1 - j <- owned plane k_begin + j
      HIPC(hipMemcpyAsync(v + plane * (g.k_begin - 1 - j), r_lo + plane * j, plane * sizeof(double),
                          hipMemcpyHostToDevice, c->stream));
    for (int j = 0; j < g.g_hi; ++j)  // ghost plane k_end + j <- owned plane k_end - 1 - j
      HIPC(hipMemcpyAsync(v + plane * (g.k_end + j), r_hi + plane * (g.g_hi - 1 - j), plane * sizeof(double),
                          hipMemcpyHostToDevice, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    return TV_OK;
  }
  if (nlo) HIPC(hipMemcpyAsync(v, r_lo, nlo * sizeof(double), hipMemcpyHostToDevice, c->stream));
  if (nhi) HIPC(hipMemcpyAsync(v + plane * g.k_end, r_hi, nhi * sizeof(double), hipMemcpyHostToDevice, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}

// the plane sends / receives of halo_grid inside an open RCCL group
static int group_planes(Ctx* c, const CgGrid& g, double* v) {
  const int64_t plane = (int64_t)g.n0 * g.n1;
  const size_t nlo = (size_t)(plane * g.g_lo), nhi = (size_t)(plane * g.g_hi);
  if (c->comm_self && g.g_lo && g.g_hi) {
    // loopback, a slab with neighbours on both sides: the neighbours are this
    // slab's own periodic images (ghost planes below <- the top owned planes,
    // ghost planes above <- the bottom ones), so the slab solves one period of
    // a y-periodic plate -- symmetric on every grid of the multigrid hierarchy
    // whose owned planes are a translate of the fine slab (tools/loopback_check.py)
    NCCLC(ncclSend(v + plane * (g.k_end - g.g_lo), nlo, ncclDouble, 0, c->comm, c->stream));
    NCCLC(ncclRecv(v, nlo, ncclDouble, 0, c->comm, c->stream));
    NCCLC(ncclSend(v + plane * g.k_begin, nhi, ncclDouble, 0, c->comm, c->stream));
    NCCLC(ncclRecv(v + plane * g.k_end, nhi, ncclDouble, 0, c->comm, c->stream));
    return TV_OK;
  }
  if (c->comm_self && (g.g_lo > 1 || g.g_hi > 1)) {
    // loopback, one neighbour, several ghost planes: the slab's MIRROR image
    // across the interface (ghost plane k_begin - 1 - j = owned plane k_begin + j),
    // the even extension about the interface midplane, whose operator on the
    // owned planes stays symmetric (a shifted copy of the boundary planes is
    // not).  One send / receive pair per plane; self pairs match in issue order.
    // (One ghost plane: the mirror is the plain copy below.)
    for (int j = 0; j < g.g_lo; ++j) {
      NCCLC(ncclSend(v + plane * (g.k_begin + j), (size_t)plane, ncclDouble, 0, c->comm, c->stream));
      NCCLC(ncclRecv(v + plane * (g.k_begin - 1 - j), (size_t)plane, ncclDouble, 0, c->comm, c->stream));
    }
    for (int j = 0; j < g.g_hi; ++j) {
      NCCLC(ncclSend(v + plane * (g.k_end - 1 - j), (size_t)plane, ncclDouble, 0, c->comm, c->stream));
      NCCLC(ncclRecv(v + plane * (g.k_end + j), (size_t)plane, ncclDouble, 0, c->comm, c->stream));
    }
    return TV_OK;
  }
  if (nlo) {  // neighbour rank - 1: send the first g_lo owned planes, receive the ghost planes below
    NCCLC(ncclSend(v + plane * g.k_begin, nlo, ncclDouble, peer(c, c->rank - 1), c->comm, c->stream));
    NCCLC(ncclRecv(v, nlo, ncclDouble, peer(c, c->rank - 1), c->comm, c->stream));
  }
  if (nhi) {
    NCCLC(ncclSend(v + plane * (g.k_end - g.g_hi), nhi, ncclDouble, peer(c, c->rank + 1), c->comm, c->stream));
    NCCLC(ncclRecv(v + plane * g.k_end, nhi, ncclDouble, peer(c, c->rank + 1), c->comm, c->stream));
  }
  return TV_OK;
}

int halo_grid(Ctx* c, const CgGrid& g, double* v) {
  if (!multi_rank(c)) return TV_OK;
  if (c->comm_stub) return stub_ghosts(c, g, v);
  if (c->host_sendrecv) return halo_host(c, g, v);
  NCCLC(ncclGroupStart());
  if (int e = group_planes(c, g, v)) return e;
  NCCLC(ncclGroupEnd());
  return TV_OK;
}

// ghosts of a partitioned unstructured mesh: pack the owned values each
// neighbour holds, then one exchange per neighbour straight into the ghost
// block that neighbour owns (ascending ranks: the host-staged pairwise
// exchanges cannot deadlock)
int halo_um(Ctx* c, double* v) {
  const int64_t nown = c->ownT_n;
  const int64_t stot = c->um_soff.empty() ? 0 : c->um_soff.back() + c->um_scnt.back();
  const int64_t rtot = c->nT - nown;
  if (c->comm_stub) {  // see stub_ghosts
    if (rtot && v != c->f[TV_F_T].ptr && v != c->f[TV_F_T_PREV].ptr)
      HIPC(hipMemsetAsync(v + nown, 0, rtot * sizeof(double), c->stream));
    return TV_OK;
  }
  launch_um_pack(c->um_sidx, stot, v, c->um_sbuf, c->stream);
  if (c->host_sendrecv) {
    double* hs = c->h_halo;
    double* hr = c->h_halo + stot;
    if (stot) HIPC(hipMemcpyAsync(hs, c->um_sbuf, stot * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    for (size_t k = 0; k < c->um_peer.size(); ++k)
      if (c->host_sendrecv(hs + c->um_soff[k], (size_t)c->um_scnt[k], c->um_peer[k], hr + c->um_roff[k],
                           (size_t)c->um_rcnt[k], c->um_peer[k], c->host_user))
        return c->fail(TV_ERR_COMM, "host sendrecv failed");
    if (rtot) HIPC(hipMemcpyAsync(v + nown, hr, rtot * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    return TV_OK;
  }
  NCCLC(ncclGroupStart());
  for (size_t k = 0; k < c->um_peer.size(); ++k) {
    if (c->um_scnt[k]) NCCLC(ncclSend(c->um_sbuf + c->um_soff[k], c->um_scnt[k], ncclDouble, peer(c, c->um_peer[k]), c->comm, c->stream));
    if (c->um_rcnt[k])
      NCCLC(ncclRecv(v + nown + c->um_roff[k], c->um_rcnt[k], ncclDouble, peer(c, c->um_peer[k]), c->comm, c->stream));
  }
  NCCLC(ncclGroupEnd());
  return TV_OK;
}

// ghost cell layers of a partitioned DG1 box (DgGrid layout): the first and
// the last owned layer, all 2^d components, packed into one buffer each; the
// neighbour's layer lands straight in the ghost region (one layer,
// component-major, as the kernels address it)
__global__ __launch_bounds__(kBlock) void k_dg_pack(const double* __restrict__ v, int64_t own, int64_t pc, int nl,
                                                    int64_t last, double* __restrict__ out) {
  const int64_t L = (int64_t)nl * pc;
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < 2 * L; t += (int64_t)gridDim.x * kBlock) {
    const int side = (int)(t / L);
    const int64_t e = t - side * L;
    const int l = (int)(e / pc);
    const int64_t q = e - (int64_t)l * pc;
    out[t] = v[(int64_t)l * own + (side ? last : 0) + q];
  }
}

int halo_dg(Ctx* c, double* v) {
  const DgGrid& g = c->dg;
  const int nl = 1 << c->dim;
  const int64_t pc = (int64_t)g.c0 * g.c1, L = (int64_t)nl * pc;
  const bool lo = g.gofs[0] >= 0, hi = g.gofs[1] >= 0;
  if (!lo && !hi) return TV_OK;
  if (c->comm_stub) {  // see stub_ghosts: the solver's ghosts read zero, the temperature keeps its ghosts
    if (v == c->f[TV_F_T].ptr || v == c->f[TV_F_T_PREV].ptr) return TV_OK;
    if (lo) HIPC(hipMemsetAsync(v + g.gofs[0], 0, L * sizeof(double), c->stream));
    if (hi) HIPC(hipMemsetAsync(v + g.gofs[1], 0, L * sizeof(double), c->stream));
    return TV_OK;
  }
  if (!c->dg_sbuf) HIPC(hipMalloc(&c->dg_sbuf, sizeof(double) * 2 * (size_t)L));
  const int nb = (int)std::min<int64_t>(1024, (2 * L + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(k_dg_pack, dim3(nb), dim3(kBlock), 0, c->stream, v, g.own, pc, nl,
                     (int64_t)(g.k_end - g.k_begin - 1) * pc, c->dg_sbuf);
  HIPC(hipGetLastError());
  if (c->host_sendrecv) {
    double* hs = c->h_halo;
    double* hr = c->h_halo + 2 * L;
    HIPC(hipMemcpyAsync(hs, c->dg_sbuf, 2 * L * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    if (lo && c->host_sendrecv(hs, (size_t)L, c->rank - 1, hr, (size_t)L, c->rank - 1, c->host_user))
      return c->fail(TV_ERR_COMM, "host sendrecv failed");
    if (hi && c->host_sendrecv(hs + L, (size_t)L, c->rank + 1, hr + L, (size_t)L, c->rank + 1, c->host_user))
      return c->fail(TV_ERR_COMM, "host sendrecv failed");
    if (lo) HIPC(hipMemcpyAsync(v + g.gofs[0], hr, L * sizeof(double), hipMemcpyHostToDevice, c->stream));
    if (hi) HIPC(hipMemcpyAsync(v + g.gofs[1], hr + L, L * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    return TV_OK;
  }
  NCCLC(ncclGroupStart());
  if (lo) {
    NCCLC(ncclSend(c->dg_sbuf, L, ncclDouble, peer(c, c->rank - 1), c->comm, c->stream));
    NCCLC(ncclRecv(v + g.gofs[0], L, ncclDouble, peer(c, c->rank - 1), c->comm, c->stream));
  }
  if (hi) {
    NCCLC(ncclSend(c->dg_sbuf + L, L, ncclDouble, peer(c, c->rank + 1), c->comm, c->stream));
    NCCLC(ncclRecv(v + g.gofs[1], L, ncclDouble, peer(c, c->rank + 1), c->comm, c->stream));
  }
  NCCLC(ncclGroupEnd());
  return TV_OK;
}

int halo(Ctx* c, double* v) {
  if (!multi_rank(c)) return TV_OK;
  if (c->fam_T == TV_DG) return halo_dg(c, v);
  if (c->um) return halo_um(c, v);
  return halo_grid(c, c->cg, v);
}

// the all-reduce of n scalars and the ghost planes of v in ONE RCCL group (one
// launch and one latency instead of two: the end of every KSPCG iteration on a
// partitioned box -- the (z.z, z.r) sums and z for the next matvec)
int allreduce_halo(Ctx* c, double* sums, int n, double* v) {
  if (!multi_rank(c)) return TV_OK;
  if (c->comm_stub || c->host_allreduce || c->um || c->fam_T != TV_CG) {
    if (int e = allreduce(c, sums, n)) return e;
    return halo(c, v);
  }
  NCCLC(ncclGroupStart());
  NCCLC(ncclAllReduce(sums, sums, n, ncclDouble, ncclSum, c->comm, c->stream));
  if (int e = group_planes(c, c->cg, v)) return e;
  NCCLC(ncclGroupEnd());
  return TV_OK;
}

// sum of a device vector over the ranks, in place (the agglomerated coarse
// levels of the partitioned multigrid: each rank contributes the coarse nodes
// its owned fine nodes restrict to, zeros elsewhere)
int allreduce_vec(Ctx* c, double* v, int64_t n) {
  if (!multi_rank(c) || n <= 0 || c->comm_stub) return TV_OK;
  if (c->host_allreduce) {
    if (c->h_big_n < (size_t)n) {
      if (c->h_big) HIPC(hipHostFree(c->h_big));
      c->h_big = nullptr;
      HIPC(hipHostMalloc(&c->h_big, sizeof(double) * (size_t)n));
      c->h_big_n = (size_t)n;
    }
    HIPC(hipMemcpyAsync(c->h_big, v, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    if (c->host_allreduce(c->h_big, (int)n, c->host_user)) return c->fail(TV_ERR_COMM, "host allreduce failed");
    HIPC(hipMemcpyAsync(v, c->h_big, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPC(hipStreamSynchronize(c->stream));  // h_big is reused by the next call
    return TV_OK;
  }
  NCCLC(ncclAllReduce(v, v, (size_t)n, ncclDouble, ncclSum, c->comm, c->stream));
  return TV_OK;
}

int allreduce(Ctx* c, double* v, int n) {
  if (!multi_rank(c) || c->comm_stub) return TV_OK;
  if (c->host_allreduce) {
    HIPC(hipMemcpyAsync(c->h_sums + 4, v, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    if (c->host_allreduce(c->h_sums + 4, n, c->host_user)) return c->fail(TV_ERR_COMM, "host allreduce failed");
    HIPC(hipMemcpyAsync(v, c->h_sums + 4, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
    return TV_OK;
  }
  NCCLC(ncclAllReduce(v, v, n, ncclDouble, ncclSum, c->comm, c->stream));
  return TV_OK;
}

// reduce partial records -> (allreduce) -> scalar logic
int reduce_logic(Ctx* c, int n, int W, int kind, int check_done) {
  if (!multi_rank(c)) {
    launch_reduce_logic(c->partials, n, W, c->sums, c->st, kind, check_done, c->stream);
  } else {
    launch_reduce_logic(c->partials, n, W, c->sums, c->st, 0, 0, c->stream);
    if (int e = allreduce(c, c->sums, W)) return e;
    if (kind) launch_logic(c->st, c->sums, kind, c->stream);
  }
  return TV_OK;
}

// ---- single-reduction PCG (Chronopoulos-Gear form, k_cgs_march) -------------
// w of the owned boundary planes + the face-workgroup facet terms (the value a
// neighbour's ghost plane must hold), packed for the halo
__global__ __launch_bounds__(kBlock) void k_cgs_pack(CgGrid g, const double* __restrict__ w,
                                                     const double* __restrict__ ff, int raxis,
                                                     double* __restrict__ out) {
  const int64_t plane = (int64_t)g.n0 * g.n1;
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < 2 * plane; t += (int64_t)gridDim.x * kBlock) {
    const int side = (int)(t / plane);
    const int64_t e = t - side * plane;
    const int k = side ? g.k_end - 1 : g.k_begin;
    const int i = (int)(e % g.n0), j = (int)(e / g.n0);
    // facet terms in the order of k_cgs_march: x face, then the row-axis face
    double fx = 0.0, fr = 0.0;
    const int fxi = (i == 0) ? 0 : (i == g.n0 - 1 ? 1 : -1);
    if (fxi >= 0 && g.ffoff[fxi] >= 0) fx = ff[g.ffoff[fxi] + j + (int64_t)g.n1 * k];
    const int c = (raxis == 1) ? j : k, n = (raxis == 1) ? g.n1 : g.n2;
    const int sd = (c == 0) ? 0 : (c == n - 1 ? 1 : -1);
    if (sd >= 0 && g.ffoff[2 * raxis + sd] >= 0) fr = ff[g.ffoff[2 * raxis + sd] + i + (int64_t)g.n0 * ((raxis == 1) ? k : j)];
    out[t] = w[e + plane * k] + (fx + fr);
  }
}

int cgs_raxis(const Ctx* c) { return (c->cg.n2 >= c->cg.n1) ? 2 : 1; }  // = plan(g).raxis

// ---- transport check (tv_comm_check) -----------------------------------------
// owned nodes of a grid level <- their global index along the level (exact in
// a double below 2^53), ghost planes <- -1
__global__ __launch_bounds__(kBlock) void k_fill_ids(double* v, int64_t plane, int64_t n, int k_begin, int k_end,
                                                     int64_t first_plane) {
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) {
    const int k = (int)(t / plane);
    v[t] = (k >= k_begin && k < k_end) ? (double)((first_plane + k) * plane + (t - (int64_t)k * plane)) : -1.0;
  }
}

namespace {
int fill_ids(Ctx* c, const CgGrid& g, double* v, int64_t first_plane) {
  const int64_t plane = (int64_t)g.n0 * g.n1, n = plane * g.n2;
  const int nb = (int)std::min<int64_t>(4096, (n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(k_fill_ids, dim3(nb), dim3(kBlock), 0, c->stream, v, plane, n, g.k_begin, g.k_end, first_plane);
  HIPC(hipGetLastError());
  return TV_OK;
}

// after an exchange of ids: the owned planes unchanged, each ghost plane holding
// the ids its neighbour sent -- the ghost's own global ids, or on a loopback
// communicator the ids of the boundary plane this rank sent itself
void check_ids(const Ctx* c, const CgGrid& g, const std::vector<double>& h, int64_t first_plane, int64_t* n_chk,
               int64_t* n_bad) {
  const int64_t plane = (int64_t)g.n0 * g.n1;
  for (int k = 0; k < g.n2; ++k) {
    int64_t src = first_plane + k;                                  // global plane the values must come from
    // loopback (group_planes): periodic images of the slab when it has both
    // neighbours, else the mirror image of its boundary planes
    const int S = g.k_end - g.k_begin;
    const bool per = g.g_lo && g.g_hi;
    if (k < g.k_begin && c->comm_self) src = first_plane + (per ? k + S : g.k_begin + (g.k_begin - 1 - k));
    if (k >= g.k_end && c->comm_self) src = first_plane + (per ? k - S : g.k_end - 1 - (k - g.k_end));
    if ((k < g.k_begin && !g.g_lo) || (k >= g.k_end && !g.g_hi)) continue;
    for (int64_t e = 0; e < plane; ++e) {
      ++*n_chk;
      if (h[(size_t)(k * plane + e)] != (double)(src * plane + e)) ++*n_bad;
    }
  }
}
}  // namespace

// Every exchange pattern the solver issues, on id-valued vectors, checked on
// the host: halo_grid (fine grid and every distributed multigrid level),
// allreduce_halo (sums + ghosts in one group), cgs_exchange (single-reduction
// form: 3 sums + packed planes), allreduce_vec (the replicated multigrid level),
// halo_um (per-neighbour groups).  Collective: every rank calls it.
int comm_check(Ctx* c, int64_t* n_chk, int64_t* n_bad) {
  *n_chk = *n_bad = 0;
  const double R = (double)c->nranks;
  const double sum_ranks = c->comm_self ? (double)(c->rank + 1) : R * (R + 1) / 2;  // sum of (rank + 1)
  const double n_contrib = c->comm_self ? 1.0 : R;
  int64_t nmax = std::max<int64_t>(c->nT, 16);
  for (const MgLevel& L : c->mg) nmax = std::max<int64_t>(nmax, L.n);
  double* v = nullptr;
  double* s = nullptr;
  double* ff = nullptr;
  HIPC(hipMalloc(&v, sizeof(double) * (size_t)nmax));
  HIPC(hipMalloc(&s, sizeof(double) * 4));
  std::vector<double> h((size_t)nmax);
  auto sums_ok = [&](const double* d, int n, const double* want) -> int {
    double hs[4];
    HIPC(hipMemcpyAsync(hs, d, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    for (int i = 0; i < n; ++i) {
      ++*n_chk;
      if (hs[i] != want[i]) ++*n_bad;
    }
    return TV_OK;
  };
  auto run = [&]() -> int {
    if (c->um) {
      const int64_t nown = c->ownT_n;
      std::vector<double> ids((size_t)c->nT, -1.0);
      for (int64_t i = 0; i < nown; ++i) ids[(size_t)i] = (double)(c->globT_off + i);
      HIPC(hipMemcpyAsync(v, ids.data(), sizeof(double) * ids.size(), hipMemcpyHostToDevice, c->stream));
      if (int e = halo_um(c, v)) return e;
      HIPC(hipMemcpyAsync(h.data(), v, sizeof(double) * (size_t)c->nT, hipMemcpyDeviceToHost, c->stream));
      HIPC(hipStreamSynchronize(c->stream));
      std::vector<int64_t> sidx(c->um_soff.empty() ? 0 : (size_t)(c->um_soff.back() + c->um_scnt.back()));
      if (!sidx.empty())
        HIPC(hipMemcpy(sidx.data(), c->um_sidx, sizeof(int64_t) * sidx.size(), hipMemcpyDeviceToHost));
      for (int64_t i = 0; i < nown; ++i) {
        ++*n_chk;
        if (h[(size_t)i] != ids[(size_t)i]) ++*n_bad;
      }
      for (size_t k = 0; k < c->um_peer.size(); ++k)
        for (int64_t j = 0; j < c->um_rcnt[k]; ++j) {
          const double got = h[(size_t)(nown + c->um_roff[k] + j)];
          ++*n_chk;
          if (c->comm_self) {  // the owned values this rank packed for "neighbour" k, in send order
            if (got != ids[(size_t)sidx[(size_t)(c->um_soff[k] + j)]]) ++*n_bad;
          } else {  // ids of the neighbour's owned vertices: outside this part's range, ascending in send order
            const bool own = got >= (double)c->globT_off && got < (double)(c->globT_off + nown);
            const bool asc = j == 0 || got > h[(size_t)(nown + c->um_roff[k] + j - 1)];
            if (got < 0 || own || !asc || got != std::floor(got)) ++*n_bad;
          }
        }
      const double hs[2] = {(double)(c->rank + 1), 1.0};
      HIPC(hipMemcpyAsync(s, hs, sizeof(hs), hipMemcpyHostToDevice, c->stream));
      if (int e = allreduce_halo(c, s, 2, v)) return e;
      const double want[2] = {sum_ranks, n_contrib};
      return sums_ok(s, 2, want);
    }
    if (c->fam_T == TV_DG) {  // ghost cell layers: global dof ids (cell-major: cell * 2^d + l)
      const DgGrid& g = c->dg;
      const int nl = 1 << c->dim;
      const int64_t pc = (int64_t)g.c0 * g.c1, L = (int64_t)nl * pc;
      const int64_t b0 = c->plane_begin, b1 = c->plane_end, nk = b1 - b0;
      std::vector<double> ids((size_t)c->nT, -1.0);
      for (int l = 0; l < nl; ++l)
        for (int64_t oc = 0; oc < g.own; ++oc) ids[(size_t)(l * g.own + oc)] = (double)((b0 * pc + oc) * nl + l);
      HIPC(hipMemcpyAsync(v, ids.data(), sizeof(double) * ids.size(), hipMemcpyHostToDevice, c->stream));
      const double hs[2] = {(double)(c->rank + 1), 1.0};
      HIPC(hipMemcpyAsync(s, hs, sizeof(hs), hipMemcpyHostToDevice, c->stream));
      if (int e = allreduce_halo(c, s, 2, v)) return e;
      const double want[2] = {sum_ranks, n_contrib};
      if (int e = sums_ok(s, 2, want)) return e;
      HIPC(hipMemcpyAsync(h.data(), v, sizeof(double) * (size_t)c->nT, hipMemcpyDeviceToHost, c->stream));
      HIPC(hipStreamSynchronize(c->stream));
      for (int64_t k = 0; k < nl * g.own; ++k) {
        ++*n_chk;
        if (h[(size_t)k] != ids[(size_t)k]) ++*n_bad;
      }
      for (int side = 0; side < 2; ++side) {
        if (g.gofs[side] < 0) continue;
        // the global layer the values must come from
        const int64_t src = c->comm_self ? (side ? b1 - 1 : b0) : (side ? b1 : b0 - 1);
        for (int l = 0; l < nl; ++l)
          for (int64_t q = 0; q < pc; ++q) {
            ++*n_chk;
            if (h[(size_t)(g.gofs[side] + l * pc + q)] != (double)((src * pc + q) * nl + l)) ++*n_bad;
          }
      }
      (void)nk;
      (void)L;
      return TV_OK;
    }
    if (c->fam_T != TV_CG) return c->fail(TV_ERR_ARG, "tv_comm_check: CG or DG temperature space");
    const CgGrid& g = c->cg;
    const int64_t first = c->plane_begin - g.k_begin;  // global plane of local plane 0
    const int64_t nloc = (int64_t)g.n0 * g.n1 * g.n2;
    auto fetch = [&](int64_t n) -> int {
      HIPC(hipMemcpyAsync(h.data(), v, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, c->stream));
      HIPC(hipStreamSynchronize(c->stream));
      return TV_OK;
    };
    // 1. halo_grid of the fine grid
    if (int e = fill_ids(c, g, v, first)) return e;
    if (int e = halo_grid(c, g, v)) return e;
    if (int e = fetch(nloc)) return e;
    check_ids(c, g, h, first, n_chk, n_bad);
    // 2. allreduce_halo: the KSPCG iteration's closing group
    if (int e = fill_ids(c, g, v, first)) return e;
    {
      const double hs[2] = {(double)(c->rank + 1), 1.0};
      HIPC(hipMemcpyAsync(s, hs, sizeof(hs), hipMemcpyHostToDevice, c->stream));
      if (int e = allreduce_halo(c, s, 2, v)) return e;
      if (int e = fetch(nloc)) return e;
      check_ids(c, g, h, first, n_chk, n_bad);
      const double want[2] = {sum_ranks, n_contrib};
      if (int e = sums_ok(s, 2, want)) return e;
    }
    // 3. cgs_exchange: the single-reduction iteration's group (facet terms zero)
    if (c->cgs && c->wsend) {
      HIPC(hipMalloc(&ff, sizeof(double) * (size_t)std::max<int64_t>(1, g.ffsize)));
      HIPC(hipMemsetAsync(ff, 0, sizeof(double) * (size_t)std::max<int64_t>(1, g.ffsize), c->stream));
      if (int e = fill_ids(c, g, v, first)) return e;
      const double hs[3] = {(double)(c->rank + 1), 1.0, 2.0};
      HIPC(hipMemcpyAsync(c->sums, hs, sizeof(hs), hipMemcpyHostToDevice, c->stream));
      if (int e = cgs_exchange(c, v, ff)) return e;
      if (int e = fetch(nloc)) return e;
      check_ids(c, g, h, first, n_chk, n_bad);
      const double want[3] = {sum_ranks, n_contrib, 2.0 * n_contrib};
      if (int e = sums_ok(c->sums, 3, want)) return e;
    }
    // 4. the distributed multigrid levels' ghost planes, the replicated level's all-reduce
    for (size_t l = 0; l < c->mg.size() && c->n_parts > 1; ++l) {
      const MgLevel& L = c->mg[l];
      const int64_t nl = (int64_t)L.g.n0 * L.g.n1 * L.g.n2;
      if (L.dist) {
        if (int e = fill_ids(c, L.g, v, L.first2)) return e;
        if (int e = halo_grid(c, L.g, v)) return e;
        if (int e = fetch(nl)) return e;
        check_ids(c, L.g, h, L.first2, n_chk, n_bad);
      } else if ((int)l + 1 == c->mg_A) {
        std::vector<double> a((size_t)nl);
        for (int64_t i = 0; i < nl; ++i) a[(size_t)i] = (double)(i % 1000) * (c->rank + 1);
        HIPC(hipMemcpyAsync(v, a.data(), sizeof(double) * (size_t)nl, hipMemcpyHostToDevice, c->stream));
        if (int e = allreduce_vec(c, v, nl)) return e;
        if (int e = fetch(nl)) return e;
        for (int64_t i = 0; i < nl; ++i) {
          ++*n_chk;
          if (h[(size_t)i] != (double)(i % 1000) * sum_ranks) ++*n_bad;
        }
      }
    }
    return TV_OK;
  };
  const int e = run();
  hipStreamSynchronize(c->stream);
  hipFree(v);
  hipFree(s);
  if (ff) hipFree(ff);
  return e;
}

// ghost planes of w_i: neighbours' packed boundary planes (RCCL group with
// the all-reduce of the iteration's sums, or the host-staged transport)
int cgs_exchange(Ctx* c, double* wout, const double* fout) {
  const CgGrid& g = c->cg;
  const int64_t plane = (int64_t)g.n0 * g.n1;
  const int blocks = (int)std::min<int64_t>(1024, (2 * plane + kBlock - 1) / kBlock);
  if (c->comm_stub) return stub_ghosts(c, g, wout);
  hipLaunchKernelGGL(k_cgs_pack, dim3(blocks), dim3(kBlock), 0, c->stream, g, wout, fout, cgs_raxis(c), c->wsend);
  if (c->host_sendrecv) {
    if (int e = allreduce(c, c->sums, 3)) return e;
    double* s_lo = c->h_halo;
    double* s_hi = c->h_halo + plane;
    double* r_lo = c->h_halo + 2 * plane;
    double* r_hi = c->h_halo + 3 * plane;
    HIPC(hipMemcpyAsync(s_lo, c->wsend, 2 * plane * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    if (g.g_lo && c->host_sendrecv(s_lo, (size_t)plane, c->rank - 1, r_lo, (size_t)plane, c->rank - 1, c->host_user))
      return c->fail(TV_ERR_COMM, "host sendrecv failed");
    if (g.g_hi && c->host_sendrecv(s_hi, (size_t)plane, c->rank + 1, r_hi, (size_t)plane, c->rank + 1, c->host_user))
      return c->fail(TV_ERR_COMM, "host sendrecv failed");
    const bool per = c->comm_self && g.g_lo && g.g_hi;  // loopback: periodic images (group_planes)
    if (g.g_lo) HIPC(hipMemcpyAsync(wout, per ? r_hi : r_lo, plane * sizeof(double), hipMemcpyHostToDevice, c->stream));
    if (g.g_hi)
      HIPC(hipMemcpyAsync(wout + plane * g.k_end, per ? r_lo : r_hi, plane * sizeof(double), hipMemcpyHostToDevice,
                          c->stream));
    return TV_OK;
  }
  // one group: the 3-scalar all-reduce and the ghost planes of w (<= 2 peers)
  NCCLC(ncclGroupStart());
  NCCLC(ncclAllReduce(c->sums, c->sums, 3, ncclDouble, ncclSum, c->comm, c->stream));
  const bool per = c->comm_self && g.g_lo && g.g_hi;  // loopback: periodic images (group_planes)
  if (g.g_lo) {
    NCCLC(ncclSend(c->wsend + (per ? plane : 0), plane, ncclDouble, peer(c, c->rank - 1), c->comm, c->stream));
    NCCLC(ncclRecv(wout, plane, ncclDouble, peer(c, c->rank - 1), c->comm, c->stream));
  }
  if (g.g_hi) {
    NCCLC(ncclSend(c->wsend + (per ? 0 : plane), plane, ncclDouble, peer(c, c->rank + 1), c->comm, c->stream));
    NCCLC(ncclRecv(wout + plane * g.k_end, plane, ncclDouble, peer(c, c->rank + 1), c->comm, c->stream));
  }
  NCCLC(ncclGroupEnd());
  return TV_OK;
}

}  // namespace tv

using namespace tv;

extern "C" {

int tv_comm_unique_id_size(void) { return (int)sizeof(ncclUniqueId); }


int tv_comm_get_unique_id(char* id_out) {
  if (!id_out) return TV_ERR_ARG;
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) {
    set_global_error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    return TV_ERR_COMM;
  }
  std::memcpy(id_out, &id, sizeof(id));
  return TV_OK;
}


int tv_comm_init(void* ctx, const char* id, int n_ranks, int rank) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !id) return TV_ERR_ARG;
  if (n_ranks != c->n_parts || rank != c->part)
    return c->fail(TV_ERR_ARG, "communicator size/rank must match the mesh partition (n_parts/part)");
  hipSetDevice(c->device);
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  NCCLC(ncclCommInitRank(&c->comm, n_ranks, uid, rank));
  c->nranks = n_ranks;
  c->rank = rank;
  // bring ghost planes of the state up to date
  if (int e = halo(c, c->f[TV_F_T].ptr)) return e;
  if (int e = halo(c, c->f[TV_F_T_PREV].ptr)) return e;
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}


int tv_comm_init_loopback(void* ctx, const char* id) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !id) return TV_ERR_ARG;
  if (c->n_parts < 2) return c->fail(TV_ERR_ARG, "tv_comm_init_loopback: a partition of a partitioned mesh only");
  if (c->comm || c->host_sendrecv || c->comm_stub) return c->fail(TV_ERR_STATE, "communicator already set");
  for (size_t k = 0; k < c->um_peer.size(); ++k)  // a self send must match its receive
    if (c->um_scnt[k] != c->um_rcnt[k])
      return c->fail(TV_ERR_ARG, "tv_comm_init_loopback: a neighbour's send and receive counts differ");
  hipSetDevice(c->device);
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  NCCLC(ncclCommInitRank(&c->comm, 1, uid, 0));
  c->nranks = c->n_parts;
  c->rank = c->part;
  c->comm_self = true;
  if (int e = halo(c, c->f[TV_F_T].ptr)) return e;
  if (int e = halo(c, c->f[TV_F_T_PREV].ptr)) return e;
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}


int tv_comm_check(void* ctx, int64_t* n_checked, int64_t* n_bad) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !n_checked || !n_bad) return TV_ERR_ARG;
  if (!multi_rank(c) || c->comm_stub)
    return c->fail(TV_ERR_STATE, "tv_comm_check: a partitioned context with a transport (not the stub)");
  hipSetDevice(c->device);
  return comm_check(c, n_checked, n_bad);
}


int tv_comm_init_host(void* ctx, int n_ranks, int rank, tv_host_allreduce_fn allreduce_fn,
                      tv_host_sendrecv_fn sendrecv_fn, void* user) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !allreduce_fn || !sendrecv_fn) return TV_ERR_ARG;
  // n_ranks = 1 on a partition of a partitioned mesh: a host-staged LOOPBACK
  // (every neighbour is this rank itself, as tv_comm_init_loopback over RCCL),
  // with the same mirrored ghost planes
  const bool self = n_ranks == 1 && rank == 0 && c->n_parts > 1;
  if (!self && (n_ranks != c->n_parts || rank != c->part))
    return c->fail(TV_ERR_ARG, "communicator size/rank must match the mesh partition (n_parts/part)");
  hipSetDevice(c->device);
  c->nranks = c->n_parts;
  c->rank = c->part;
  c->comm_self = self;
  c->host_allreduce = allreduce_fn;
  c->host_sendrecv = sendrecv_fn;
  c->host_user = user;
  if (c->um) {  // the packed sends, then the ghosts
    const int64_t stot = c->um_soff.empty() ? 0 : c->um_soff.back() + c->um_scnt.back();
    HIPC(hipHostMalloc(&c->h_halo, sizeof(double) * (size_t)std::max<int64_t>(1, stot + c->nT - c->ownT_n)));
  } else if (c->fam_T == TV_CG) {  // send + receive blocks of g_lo + g_hi planes
    const int64_t plane = (int64_t)c->cg.n0 * c->cg.n1;
    HIPC(hipHostMalloc(&c->h_halo, sizeof(double) * 2 * (size_t)plane * std::max(2, c->cg.g_lo + c->cg.g_hi)));
  } else {  // DG: 2 send + 2 receive cell layers of 2^d components
    const int64_t L = ((int64_t)1 << c->dim) * c->dg.c0 * c->dg.c1;
    HIPC(hipHostMalloc(&c->h_halo, sizeof(double) * 4 * (size_t)L));
  }
  if (int e = halo(c, c->f[TV_F_T].ptr)) return e;
  if (int e = halo(c, c->f[TV_F_T_PREV].ptr)) return e;
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}


int tv_comm_init_stub(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  if (c->n_parts < 2) return c->fail(TV_ERR_ARG, "tv_comm_init_stub: a partition of a partitioned mesh only");
  if (c->O.ksp_fixed_its <= 0)  // measurement only: its decoupled solve is no solution
    return c->fail(TV_ERR_ARG, "tv_comm_init_stub: measurement only, needs options.ksp_fixed_its > 0");
  hipSetDevice(c->device);
  c->nranks = c->n_parts;
  c->rank = c->part;
  c->comm_stub = true;
  if (int e = halo(c, c->f[TV_F_T].ptr)) return e;
  if (int e = halo(c, c->f[TV_F_T_PREV].ptr)) return e;
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}


int tv_comm_time(void* ctx, int pattern, int reps, double* us_per_call) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !us_per_call || reps < 1 || pattern < 0 || pattern >= TV_XCHG_COUNT) return TV_ERR_ARG;
  if (!multi_rank(c)) return c->fail(TV_ERR_STATE, "tv_comm_time: a partitioned context with a transport");
  if (c->um || c->fam_T != TV_CG) return c->fail(TV_ERR_ARG, "tv_comm_time: partitioned CG1 box meshes");
  hipSetDevice(c->device);
  // the multigrid level a pattern needs (distributed level 1 / 2, the replicated level mg_A)
  MgLevel* lev = nullptr;
  if (pattern == TV_XCHG_VEC) {
    if (!c->mg_on || c->mg_A < 1 || (size_t)c->mg_A > c->mg.size()) return TV_ERR_ARG;
    lev = &c->mg[(size_t)c->mg_A - 1];
  } else if (pattern == TV_XCHG_HALO_L1 || pattern == TV_XCHG_HALO_L2) {
    const size_t l = pattern == TV_XCHG_HALO_L1 ? 1 : 2;
    if (!c->mg_on || c->mg.size() < l || !c->mg[l - 1].dist) return TV_ERR_ARG;
    lev = &c->mg[l - 1];
  }
  auto once = [&]() -> int {
    switch (pattern) {
      case TV_XCHG_HALO: return halo_grid(c, c->cg, c->w);
      case TV_XCHG_ALLREDUCE1: return allreduce(c, c->sums + 4, 1);
      case TV_XCHG_CLOSE: return allreduce_halo(c, c->sums + 4, 2, c->w);
      case TV_XCHG_VEC: return allreduce_vec(c, lev->b, lev->n);
      default: return halo_grid(c, lev->g, lev->x);
    }
  };
  if (int e = once()) return e;  // warm-up (RCCL connects its peers at the first use)
  hipEvent_t e0, e1;
  HIPC(hipEventCreate(&e0));
  HIPC(hipEventCreate(&e1));
  HIPC(hipStreamSynchronize(c->stream));
  HIPC(hipEventRecord(e0, c->stream));
  for (int r = 0; r < reps; ++r)
    if (int e = once()) return e;
  HIPC(hipEventRecord(e1, c->stream));
  HIPC(hipEventSynchronize(e1));
  float ms = 0.f;
  HIPC(hipEventElapsedTime(&ms, e0, e1));
  HIPC(hipEventDestroy(e0));
  HIPC(hipEventDestroy(e1));
  *us_per_call = 1e3 * (double)ms / reps;
  return TV_OK;
}


int tv_halo_exchange(void* ctx, int field) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || field < 0 || field >= TV_NUM_FIELDS || !c->f[field].ptr) return TV_ERR_ARG;
  if (c->f[field].space != 0 || c->f[field].bs != 1) return c->fail(TV_ERR_ARG, "halo exchange: scalar T-space fields only");
  if (int e = halo(c, c->f[field].ptr)) return e;
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}

}  // extern "C"
