// Micro-benchmark: the 27-point tensor-product J x of the C4 grid (401 x 51 x
// 401 nodes, x fastest) as a march (the library's design: one barrier per
// plane, loads two planes ahead) against "cube" tiles that load their whole
// (TZ + 2) x (TY + 2) row block into LDS up front -- every load of the tile in
// flight at once, ONE barrier -- and then sweep the planes from LDS.
//   hipcc -O3 --offload-arch=gfx950 cube_probe.hip -o cube_probe; ./cube_probe f
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

constexpr int W = 64, SEG = 62;

__device__ __forceinline__ double shr1(double v) {
  int lo = __double2loint(v), hi = __double2hiint(v);
  lo = __builtin_amdgcn_update_dpp(0, lo, 0x138, 0xF, 0xF, false);
  hi = __builtin_amdgcn_update_dpp(0, hi, 0x138, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double shl1(double v) {
  int lo = __double2loint(v), hi = __double2hiint(v);
  lo = __builtin_amdgcn_update_dpp(0, lo, 0x130, 0xF, 0xF, false);
  hi = __builtin_amdgcn_update_dpp(0, hi, 0x130, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

struct Grid { int n0, nQ, nR; long sQ, sR; };  // Q: plane axis of the tiles' sweep, R: row axis
__constant__ double cM[3] = {1.0 / 6, 2.0 / 3, 1.0 / 6};
__constant__ double cK[3] = {-1.0, 2.0, -1.0};

__device__ __forceinline__ int remap(int b, int nb) {  // XCD-contiguous shares of the block sequence
  const int q = nb / 8, r = nb % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// one output row of a sweep: sliding z window of (us, vs) = (My, Ky) row stencils
struct Win {
  double us_m = 0, us_c = 0, vs_m = 0, vs_c = 0;
  __device__ __forceinline__ double push(double x0, double x1, double x2, bool emit) {
    const double da = 0.1;
    const double us_p = cM[0] * x0 + cM[1] * x1 + cM[2] * x2;
    const double vs_p = cK[0] * x0 + cK[1] * x1 + cK[2] * x2;
    double y = 0.0;
    if (emit) {
      const double S1 = cM[0] * (us_m + da * vs_m) + cM[1] * (us_c + da * vs_c) + cM[2] * (us_p + da * vs_p) +
                        da * (cK[0] * us_m + cK[1] * us_c + cK[2] * us_p);
      const double S2 = da * (cM[0] * us_m + cM[1] * us_c + cM[2] * us_p);
      y = cM[0] * shr1(S1) + cM[1] * S1 + cM[2] * shl1(S1) + cK[0] * shr1(S2) + cK[1] * S2 + cK[2] * shl1(S2);
    }
    us_m = us_c; us_c = us_p; vs_m = vs_c; vs_c = vs_p;
    return y;
  }
};

// ---------------- A: the march (LDS slab, one barrier per plane, PF 2) --------
template <int R>
__global__ __launch_bounds__(R * W) void kA(Grid g, const double* __restrict__ in, double* __restrict__ out,
                                            int nseg, int qchunk) {
  __shared__ double lds[2][R + 2][W];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nrb = (g.nR + R - 1) / R;
  const int b = remap(blockIdx.x, gridDim.x);
  const int seg = b % nseg, t = b / nseg, rb = t % nrb, chunk = t / nrb;
  const int r0 = rb * R, r = r0 + wave;
  const int q0 = chunk * qchunk, q1 = min(q0 + qchunk, g.nQ);
  const int i = seg * SEG - 1 + lane;
  const bool col_ok = i >= 0 && i < g.n0;
  const bool writer = col_ok && lane >= 1 && lane <= SEG && r < g.nR;
  const bool halo = wave == 0 || wave == R - 1;
  const int hrow = wave == 0 ? r0 - 1 : (wave == R - 1 ? r0 + R : r);
  const int hslot = wave == 0 ? 0 : R + 1;
  auto okf = [&](int rr, int L) { return col_ok && rr >= 0 && rr < g.nR && L >= 0 && L < g.nQ; };
  auto fetch = [&](int rr, int L) { return in[okf(rr, L) ? (long)i + g.sR * rr + g.sQ * L : 0]; };
  double a = fetch(r, q0 - 1), ah = fetch(hrow, q0 - 1);
  double bb = fetch(r, q0), bh = fetch(hrow, q0);
  double c, ch;
  Win win;
  auto step = [&](int L, double v, double hv) {
    const int buf = L & 1;
    lds[buf][wave + 1][lane] = okf(r, L) ? v : 0.0;
    if (halo) lds[buf][hslot][lane] = okf(hrow, L) ? hv : 0.0;
    __syncthreads();
    const bool emit = L >= q0 + 1 && L <= q1;
    const double y = win.push(lds[buf][wave][lane], lds[buf][wave + 1][lane], lds[buf][wave + 2][lane], emit);
    if (emit && writer) out[(long)i + g.sR * r + g.sQ * (L - 1)] = y;
  };
  for (int L = q0 - 1; L <= q1; L += 3) {
    c = fetch(r, L + 2); ch = fetch(hrow, L + 2);
    step(L, a, ah);
    a = fetch(r, L + 3); ah = fetch(hrow, L + 3);
    step(L + 1, bb, bh);
    bb = fetch(r, L + 4); bh = fetch(hrow, L + 4);
    step(L + 2, c, ch);
  }
}

// ---------------- E: cube tile, everything loaded before one barrier ----------
// TY waves (one output row each) x TZ planes x 62 x-nodes; LDS [TZ + 2][TY + 2][64]
template <int TY, int TZ>
__global__ __launch_bounds__(TY * W) void kE(Grid g, const double* __restrict__ in, double* __restrict__ out,
                                             int nseg, int nrb) {
  __shared__ double s[TZ + 2][TY + 2][W];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = remap(blockIdx.x, gridDim.x);
  const int seg = b % nseg, t = b / nseg, rb = t % nrb, zb = t / nrb;
  const int r0 = rb * TY, z0 = zb * TZ;
  const int i = seg * SEG - 1 + lane;
  const bool col_ok = i >= 0 && i < g.n0;
  constexpr int NROWS = (TZ + 2) * (TY + 2);
  constexpr int PER = (NROWS + TY - 1) / TY;
  double v[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = wave + k * TY;
    const int zz = e / (TY + 2), yy = e % (TY + 2);
    const int gz = z0 - 1 + zz, gy = r0 - 1 + yy;
    const bool ok = e < NROWS && col_ok && gz >= 0 && gz < g.nQ && gy >= 0 && gy < g.nR;
    v[k] = ok ? in[(long)i + g.sR * gy + g.sQ * gz] : 0.0;
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = wave + k * TY;
    if (e < NROWS) s[e / (TY + 2)][e % (TY + 2)][lane] = v[k];
  }
  __syncthreads();
  const int r = r0 + wave;
  const bool writer = col_ok && lane >= 1 && lane <= SEG && r < g.nR;
  Win win;
#pragma unroll
  for (int zz = 0; zz < TZ + 2; ++zz) {
    const bool emit = zz >= 2;
    const double y = win.push(s[zz][wave][lane], s[zz][wave + 1][lane], s[zz][wave + 2][lane], emit);
    const int gz = z0 + zz - 2;
    if (emit && writer && gz < g.nQ) out[(long)i + g.sR * r + g.sQ * gz] = y;
  }
}

// ---------------- F: cube tile with two output rows per wave -----------------
template <int TY, int TZ>
__global__ __launch_bounds__(TY / 2 * W) void kF(Grid g, const double* __restrict__ in, double* __restrict__ out,
                                                 int nseg, int nrb) {
  constexpr int NW = TY / 2;
  __shared__ double s[TZ + 2][TY + 2][W];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = remap(blockIdx.x, gridDim.x);
  const int seg = b % nseg, t = b / nseg, rb = t % nrb, zb = t / nrb;
  const int r0 = rb * TY, z0 = zb * TZ;
  const int i = seg * SEG - 1 + lane;
  const bool col_ok = i >= 0 && i < g.n0;
  constexpr int NROWS = (TZ + 2) * (TY + 2);
  constexpr int PER = (NROWS + NW - 1) / NW;
  double v[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = wave + k * NW;
    const int zz = e / (TY + 2), yy = e % (TY + 2);
    const int gz = z0 - 1 + zz, gy = r0 - 1 + yy;
    const bool ok = e < NROWS && col_ok && gz >= 0 && gz < g.nQ && gy >= 0 && gy < g.nR;
    v[k] = ok ? in[(long)i + g.sR * gy + g.sQ * gz] : 0.0;
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = wave + k * NW;
    if (e < NROWS) s[e / (TY + 2)][e % (TY + 2)][lane] = v[k];
  }
  __syncthreads();
  const int ra = r0 + 2 * wave;
  Win wa, wb;
#pragma unroll
  for (int zz = 0; zz < TZ + 2; ++zz) {
    const bool emit = zz >= 2;
    const double x0 = s[zz][2 * wave][lane], x1 = s[zz][2 * wave + 1][lane], x2 = s[zz][2 * wave + 2][lane],
                 x3 = s[zz][2 * wave + 3][lane];
    const double ya = wa.push(x0, x1, x2, emit), yb = wb.push(x1, x2, x3, emit);
    const int gz = z0 + zz - 2;
    if (emit && col_ok && lane >= 1 && lane <= SEG && gz < g.nQ) {
      if (ra < g.nR) out[(long)i + g.sR * ra + g.sQ * gz] = ya;
      if (ra + 1 < g.nR) out[(long)i + g.sR * (ra + 1) + g.sQ * gz] = yb;
    }
  }
}


// ---------------- R: the march's read pattern alone (no LDS, no compute) ------
// every wave streams its row over the chunk's planes (+ halo planes; halo waves
// their halo rows too) and sums; ALIGN: 64-node segments starting on 512 B
// (i = 64 seg + lane) instead of the march's 62-output segments with one halo
// lane either side (i = 62 seg - 1 + lane, a 5th 128 B line per row)
template <int R, bool ALIGN, bool HALO>
__global__ __launch_bounds__(R * W) void kR(Grid g, const double* __restrict__ in, double* __restrict__ out,
                                            int nseg, int qchunk) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nrb = (g.nR + R - 1) / R;
  const int b = remap(blockIdx.x, gridDim.x);
  const int seg = b % nseg, t = b / nseg, rb = t % nrb, chunk = t / nrb;
  const int r0 = rb * R, r = r0 + wave;
  const int q0 = chunk * qchunk, q1 = min(q0 + qchunk, g.nQ);
  const int i = ALIGN ? seg * 64 + lane : seg * SEG - 1 + lane;
  const bool col_ok = i >= 0 && i < g.n0;
  const bool halo = HALO && (wave == 0 || wave == R - 1);
  const int hrow = wave == 0 ? r0 - 1 : r0 + R;
  double acc = 0.0;
  const int L0 = HALO ? q0 - 1 : q0, L1 = HALO ? q1 + 1 : q1;
#pragma unroll 4
  for (int L = L0; L < L1; ++L) {
    const bool ok = col_ok && r < g.nR && L >= 0 && L < g.nQ;
    acc += in[ok ? (long)i + g.sR * r + g.sQ * L : 0];
    if (halo) {
      const bool okh = col_ok && hrow >= 0 && hrow < g.nR && L >= 0 && L < g.nQ;
      acc += in[okh ? (long)i + g.sR * hrow + g.sQ * L : 0];
    }
  }
  if (col_ok && r < g.nR) out[(long)i + g.sR * r] = acc;
}

// ---------------- R-BAL: the same reads, halo rows spread over every wave -----
// planes in groups of G = R / 2: per group each wave loads its own row on the
// G planes and ONE of the 2 G halo row-planes, so no wave carries twice the loads
template <int R>
__global__ __launch_bounds__(R * W) void kRB(Grid g, const double* __restrict__ in, double* __restrict__ out,
                                             int nseg, int qchunk) {
  constexpr int G = R / 2;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nrb = (g.nR + R - 1) / R;
  const int b = remap(blockIdx.x, gridDim.x);
  const int seg = b % nseg, t = b / nseg, rb = t % nrb, chunk = t / nrb;
  const int r0 = rb * R, r = r0 + wave;
  const int q0 = chunk * qchunk, q1 = min(q0 + qchunk, g.nQ);
  const int i = seg * SEG - 1 + lane;
  const bool col_ok = i >= 0 && i < g.n0;
  const int hr = (wave & 1) ? r0 + R : r0 - 1, hq = wave >> 1;
  double acc = 0.0;
  for (int P = q0 - 1; P <= q1; P += G) {
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const int L = P + k;
      const bool ok = col_ok && r < g.nR && L >= 0 && L < g.nQ && L <= q1;
      acc += in[ok ? (long)i + g.sR * r + g.sQ * L : 0];
    }
    const int L = P + hq;
    const bool okh = col_ok && hr >= 0 && hr < g.nR && L >= 0 && L < g.nQ && L <= q1;
    acc += in[okh ? (long)i + g.sR * hr + g.sQ * L : 0];
  }
  if (col_ok && r < g.nR) out[(long)i + g.sR * r] = acc;
}

// ---------------- AB: the march with balanced halo loads ---------------------
// G = R / 2 planes per barrier step; per step every wave loads its own row on
// the G planes and one of the 2 G halo row-planes (loads of the next step in
// flight while this one is computed); LDS [2][G][R + 2][64]
template <int R>
__global__ __launch_bounds__(R * W) void kAB(Grid g, const double* __restrict__ in, double* __restrict__ out,
                                             int nseg, int qchunk) {
  constexpr int G = R / 2;
  __shared__ double lds[2][G][R + 2][W];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nrb = (g.nR + R - 1) / R;
  const int b = remap(blockIdx.x, gridDim.x);
  const int seg = b % nseg, t = b / nseg, rb = t % nrb, chunk = t / nrb;
  const int r0 = rb * R, r = r0 + wave;
  const int q0 = chunk * qchunk, q1 = min(q0 + qchunk, g.nQ);
  const int i = seg * SEG - 1 + lane;
  const bool col_ok = i >= 0 && i < g.n0;
  const bool writer = col_ok && lane >= 1 && lane <= SEG && r < g.nR;
  const int hr = (wave & 1) ? r0 + R : r0 - 1, hq = wave >> 1, hslot = (wave & 1) ? R + 1 : 0;
  auto okf = [&](int rr, int L) { return col_ok && rr >= 0 && rr < g.nR && L >= 0 && L < g.nQ && L <= q1; };
  auto fetch = [&](int rr, int L) { return in[okf(rr, L) ? (long)i + g.sR * rr + g.sQ * L : 0]; };
  double own[2][G], hv[2];
  auto load = [&](int s, int P) {
#pragma unroll
    for (int k = 0; k < G; ++k) own[s][k] = fetch(r, P + k);
    hv[s] = fetch(hr, P + hq);
  };
  Win win;
  auto step = [&](const int s, int P) {  // s: a literal 0 / 1 (static register indices after inlining)
    if (P + G <= q1) load(s ^ 1, P + G);
#pragma unroll
    for (int k = 0; k < G; ++k) lds[s][k][wave + 1][lane] = okf(r, P + k) ? own[s][k] : 0.0;
    lds[s][hq][hslot][lane] = okf(hr, P + hq) ? hv[s] : 0.0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const int L = P + k;
      const bool emit = L >= q0 + 1 && L <= q1;
      const double y = win.push(lds[s][k][wave][lane], lds[s][k][wave + 1][lane], lds[s][k][wave + 2][lane], emit);
      if (emit && writer) out[(long)i + g.sR * r + g.sQ * (L - 1)] = y;
    }
  };
  int P = q0 - 1;
  load(0, P);
  for (; P <= q1; P += 2 * G) {
    step(0, P);
    if (P + G > q1) break;
    step(1, P + G);
  }
}

// ---------------- A2 / AB2: the fused-PCG shape (two inputs z, p_old; p = z + b p_old stored)
template <int R, bool BAL>
__global__ __launch_bounds__(R * W) void kF2(Grid g, const double* __restrict__ z, const double* __restrict__ po,
                                             double* __restrict__ pn, double* __restrict__ out, int nseg, int qchunk) {
  constexpr int G = BAL ? R / 2 : 1;
  __shared__ double lds[2][G][R + 2][W];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nrb = (g.nR + R - 1) / R;
  const int b = remap(blockIdx.x, gridDim.x);
  const int seg = b % nseg, t = b / nseg, rb = t % nrb, chunk = t / nrb;
  const int r0 = rb * R, r = r0 + wave;
  const int q0 = chunk * qchunk, q1 = min(q0 + qchunk, g.nQ);
  const int i = seg * SEG - 1 + lane;
  const bool col_ok = i >= 0 && i < g.n0;
  const bool writer = col_ok && lane >= 1 && lane <= SEG && r < g.nR;
  const double beta = 0.37;
  // halo row-planes: BAL -> one per wave per group; else waves 0 / R-1 on every plane
  const int hr = BAL ? ((wave & 1) ? r0 + R : r0 - 1) : (wave == 0 ? r0 - 1 : r0 + R);
  const int hq = BAL ? (wave >> 1) : 0, hslot = BAL ? ((wave & 1) ? R + 1 : 0) : (wave == 0 ? 0 : R + 1);
  const bool hload = BAL || wave == 0 || wave == R - 1;
  auto okf = [&](int rr, int L) { return col_ok && rr >= 0 && rr < g.nR && L >= 0 && L < g.nQ && L <= q1; };
  auto off = [&](int rr, int L) { return okf(rr, L) ? (long)i + g.sR * rr + g.sQ * L : 0L; };
  double oz[2][G], op[2][G], hz[2], hp[2];
  auto load = [&](int s, int P) {
#pragma unroll
    for (int k = 0; k < G; ++k) { const long o = off(r, P + k); oz[s][k] = z[o]; op[s][k] = po[o]; }
    if (hload) { const long o = off(hr, P + hq); hz[s] = z[o]; hp[s] = po[o]; }
  };
  Win win;
  auto step = [&](const int s, int P) {
    if (P + G <= q1) load(s ^ 1, P + G);
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const int L = P + k;
      const double pv = oz[s][k] + beta * op[s][k];
      if (writer && L >= q0 && L < q1) pn[(long)i + g.sR * r + g.sQ * L] = pv;
      lds[s][k][wave + 1][lane] = okf(r, L) ? pv : 0.0;
    }
    if (hload) lds[s][hq][hslot][lane] = okf(hr, P + hq) ? hz[s] + beta * hp[s] : 0.0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const int L = P + k;
      const bool emit = L >= q0 + 1 && L <= q1;
      const double y = win.push(lds[s][k][wave][lane], lds[s][k][wave + 1][lane], lds[s][k][wave + 2][lane], emit);
      if (emit && writer) out[(long)i + g.sR * r + g.sQ * (L - 1)] = y;
    }
  };
  int P = q0 - 1;
  load(0, P);
  if (BAL) {
    for (; P <= q1; P += 2 * G) {
      step(0, P);
      if (P + G > q1) break;
      step(1, P + G);
    }
  } else {  // one plane per step, prefetch one step ahead (the library's PF 2 is one more)
    for (; P <= q1; P += 2) {
      step(0, P);
      if (P + 1 > q1) break;
      step(1, P + 1);
    }
  }
}

__global__ void copy1(const double* __restrict__ a, double* __restrict__ b, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) b[i] = a[i];
}
__global__ void flushk(double* p, long n) {  // read-only sweep: evicts the inputs, leaves no dirty lines
  double acc = 0.0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) acc += p[i];
  if (acc == 12345.678) p[0] = acc;
}
double* g_flush = nullptr;
bool g_do_flush = false;
template <typename F>
float timeit(F f, int reps, hipEvent_t e0, hipEvent_t e1) {
  if (g_do_flush) {
    std::vector<float> v;
    f();
    for (int k = 0; k < reps; ++k) {
      flushk<<<4096, 256>>>(g_flush, (1L << 30) / 8);
      CK(hipEventRecord(e0));
      f();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.push_back(ms);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2] * 1e3f;  // median, us
  }
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int k = 0; k < reps; ++k) f();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

int main(int argc, char** argv) {
  Grid g{401, 51, 401, 401, 401L * 51};
  const long N = (long)g.n0 * g.nQ * g.nR;
  double *x, *y, *fl;
  CK(hipMalloc(&x, N * 8));
  CK(hipMalloc(&y, N * 8));
  CK(hipMalloc(&fl, 1L << 30));
  CK(hipMemset(fl, 0, 1L << 30));
  g_flush = fl;
  g_do_flush = argc > 1 && argv[1][0] == 'f';
  printf("inputs %s\n", g_do_flush ? "HBM-resident (1 GB read sweep before each rep, median)" : "warm (back-to-back)");
  std::vector<double> h(N);
  for (long k = 0; k < N; ++k) h[k] = 1.0 + 1e-3 * (k % 977) + 1e-6 * (k % 131);
  CK(hipMemcpy(x, h.data(), N * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 31;
  const double bytes = 16.0 * N;
  const int nseg = (g.n0 + SEG - 1) / SEG;
  auto rep = [&](const char* name, float us, int blocks) {
    printf("%-36s %8.2f us  %7.1f GB/s  blocks %d\n", name, us, bytes / (us * 1e-6) / 1e9, blocks);
  };
  rep("copy (8 B / lane)", timeit([&] { copy1<<<4096, 256>>>(x, y, N); }, reps, e0, e1), 4096);
  std::vector<double> ya(N), yb(N);
  {  // the march, 4 chunks of 13 planes (the production C4 shape)
    const int nrb = (g.nR + 7) / 8, qc = 13, nb = nseg * nrb * ((g.nQ + qc - 1) / qc);
    rep("A march R=8 qchunk=13", timeit([&] { kA<8><<<nb, 8 * W>>>(g, x, y, nseg, qc); }, reps, e0, e1), nb);
    CK(hipMemset(y, 0, N * 8));
    kA<8><<<nb, 8 * W>>>(g, x, y, nseg, qc);
    CK(hipMemcpy(ya.data(), y, N * 8, hipMemcpyDeviceToHost));
  }
  auto check = [&](const char* nm) {
    CK(hipMemcpy(yb.data(), y, N * 8, hipMemcpyDeviceToHost));
    double md = 0;
    for (long k = 0; k < N; ++k) md = fmax(md, fabs(ya[k] - yb[k]));
    printf("   %s: max |A - this| = %g\n", nm, md);
  };
#define RUN_E(TY, TZ)                                                                                     \
  {                                                                                                       \
    const int nrb = (g.nR + TY - 1) / TY, nzb = (g.nQ + TZ - 1) / TZ, nb = nseg * nrb * nzb;              \
    char nm[64];                                                                                          \
    snprintf(nm, sizeof nm, "E cube TY=%d TZ=%d", TY, TZ);                                                \
    rep(nm, timeit([&] { kE<TY, TZ><<<nb, TY * W>>>(g, x, y, nseg, nrb); }, reps, e0, e1), nb);            \
    CK(hipMemset(y, 0, N * 8));                                                                           \
    kE<TY, TZ><<<nb, TY * W>>>(g, x, y, nseg, nrb);                                                       \
    check(nm);                                                                                            \
  }
#define RUN_F(TY, TZ)                                                                                     \
  {                                                                                                       \
    const int nrb = (g.nR + TY - 1) / TY, nzb = (g.nQ + TZ - 1) / TZ, nb = nseg * nrb * nzb;              \
    char nm[64];                                                                                          \
    snprintf(nm, sizeof nm, "F cube 2 rows/wave TY=%d TZ=%d", TY, TZ);                                    \
    rep(nm, timeit([&] { kF<TY, TZ><<<nb, TY / 2 * W>>>(g, x, y, nseg, nrb); }, reps, e0, e1), nb);        \
    CK(hipMemset(y, 0, N * 8));                                                                           \
    kF<TY, TZ><<<nb, TY / 2 * W>>>(g, x, y, nseg, nrb);                                                   \
    check(nm);                                                                                            \
  }
  {  // the march with the axes swapped: rows along storage axis 1 (51 rows, adjacent in memory: a tile's
     // rows of one plane are one contiguous run), the march along storage axis 2 (401 planes)
    Grid h{401, 401, 51, 401L * 51, 401};
    for (int qc : {13, 16, 26, 51}) {
      const int nrb = (h.nR + 7) / 8, nb = nseg * nrb * ((h.nQ + qc - 1) / qc);
      char nm[64];
      snprintf(nm, sizeof nm, "A swapped R=8 qchunk=%d", qc);
      rep(nm, timeit([&] { kA<8><<<nb, 8 * W>>>(h, x, y, nseg, qc); }, reps, e0, e1), nb);
    }
    for (int qc : {16, 26}) {
      const int nrb = (h.nR + 3) / 4, nb = nseg * nrb * ((h.nQ + qc - 1) / qc);
      char nm[64];
      snprintf(nm, sizeof nm, "A swapped R=4 qchunk=%d", qc);
      rep(nm, timeit([&] { kA<4><<<nb, 4 * W>>>(h, x, y, nseg, qc); }, reps, e0, e1), nb);
    }
    const int qc = 16, nrb = (h.nR + 7) / 8, nb = nseg * nrb * ((h.nQ + qc - 1) / qc);
    CK(hipMemset(y, 0, N * 8));
    kA<8><<<nb, 8 * W>>>(h, x, y, nseg, qc);
    check("A swapped R=8 qchunk=16");
    {
      const int TY = 8, TZ = 13, nrbE = (h.nR + TY - 1) / TY, nzb = (h.nQ + TZ - 1) / TZ, nbE = nseg * nrbE * nzb;
      rep("E swapped TY=8 TZ=13", timeit([&] { kE<8, 13><<<nbE, 8 * W>>>(h, x, y, nseg, nrbE); }, reps, e0, e1), nbE);
    }
  }
  {
    const int nrb = (g.nR + 7) / 8, qc = 13, nch = (g.nQ + qc - 1) / qc;
    const int nsegA = (g.n0 + 63) / 64;
    rep("R reads march-shaped (62-seg, halos)", timeit([&] { kR<8, false, true><<<nseg * nrb * nch, 8 * W>>>(g, x, y, nseg, qc); }, reps, e0, e1), nseg * nrb * nch);
    rep("R reads 62-seg, no halos", timeit([&] { kR<8, false, false><<<nseg * nrb * nch, 8 * W>>>(g, x, y, nseg, qc); }, reps, e0, e1), nseg * nrb * nch);
    rep("R reads aligned 64-seg, halos", timeit([&] { kR<8, true, true><<<nsegA * nrb * nch, 8 * W>>>(g, x, y, nsegA, qc); }, reps, e0, e1), nsegA * nrb * nch);
    rep("R reads aligned 64-seg, no halos", timeit([&] { kR<8, true, false><<<nsegA * nrb * nch, 8 * W>>>(g, x, y, nsegA, qc); }, reps, e0, e1), nsegA * nrb * nch);
    rep("R-BAL reads, halos spread R=8", timeit([&] { kRB<8><<<nseg * nrb * nch, 8 * W>>>(g, x, y, nseg, qc); }, reps, e0, e1), nseg * nrb * nch);
    rep("R-BAL reads, halos spread R=4", timeit([&] { kRB<4><<<nseg * ((g.nR + 3) / 4) * nch, 4 * W>>>(g, x, y, nseg, qc); }, reps, e0, e1), nseg * ((g.nR + 3) / 4) * nch);
    for (int qcb : {13, 16, 26}) {
      const int nchb = (g.nQ + qcb - 1) / qcb;
      char nm[64];
      snprintf(nm, sizeof nm, "AB march balanced R=8 qchunk=%d", qcb);
      rep(nm, timeit([&] { kAB<8><<<nseg * nrb * nchb, 8 * W>>>(g, x, y, nseg, qcb); }, reps, e0, e1), nseg * nrb * nchb);
      CK(hipMemset(y, 0, N * 8));
      kAB<8><<<nseg * nrb * nchb, 8 * W>>>(g, x, y, nseg, qcb);
      check(nm);
    }
    {
      const int nrb4 = (g.nR + 3) / 4;
      rep("AB march balanced R=4 qchunk=13", timeit([&] { kAB<4><<<nseg * nrb4 * nch, 4 * W>>>(g, x, y, nseg, qc); }, reps, e0, e1), nseg * nrb4 * nch);
      CK(hipMemset(y, 0, N * 8));
      kAB<4><<<nseg * nrb4 * nch, 4 * W>>>(g, x, y, nseg, qc);
      check("AB R=4");
      const int nrb16 = (g.nR + 15) / 16;
      rep("AB march balanced R=16 qchunk=13", timeit([&] { kAB<16><<<nseg * nrb16 * nch, 16 * W>>>(g, x, y, nseg, qc); }, reps, e0, e1), nseg * nrb16 * nch);
    }
    {  // fused-PCG shape: reads z and p_old, writes p and w (32 B per node)
      double *z2, *pn;
      CK(hipMalloc(&z2, N * 8));
      CK(hipMalloc(&pn, N * 8));
      CK(hipMemcpy(z2, x, N * 8, hipMemcpyDeviceToDevice));
      auto rep2 = [&](const char* name, float us, int blocks) {
        printf("%-36s %8.2f us  %7.1f GB/s (32 B/node)  blocks %d\n", name, us, 32.0 * N / (us * 1e-6) / 1e9, blocks);
      };
      for (int qcb : {13, 26}) {
        const int nchb = (g.nQ + qcb - 1) / qcb;
        char nm[64];
        snprintf(nm, sizeof nm, "F2 fused shape, halos on 2 waves q=%d", qcb);
        rep2(nm, timeit([&] { kF2<8, false><<<nseg * nrb * nchb, 8 * W>>>(g, z2, x, pn, y, nseg, qcb); }, reps, e0, e1), nseg * nrb * nchb);
        snprintf(nm, sizeof nm, "F2 fused shape, balanced q=%d", qcb);
        rep2(nm, timeit([&] { kF2<8, true><<<nseg * nrb * nchb, 8 * W>>>(g, z2, x, pn, y, nseg, qcb); }, reps, e0, e1), nseg * nrb * nchb);
      }
      CK(hipFree(z2));
      CK(hipFree(pn));
    }
    rep("R reads aligned, 1 chunk (51 planes)", timeit([&] { kR<8, true, false><<<nsegA * nrb, 8 * W>>>(g, x, y, nsegA, 51); }, reps, e0, e1), nsegA * nrb);
  }
  RUN_E(4, 13)
  RUN_E(4, 17)
  RUN_E(4, 26)
  RUN_E(8, 9)
  RUN_E(8, 13)
  RUN_E(2, 17)
  RUN_E(2, 26)
  RUN_F(4, 13)
  RUN_F(8, 13)
  RUN_F(8, 9)
  RUN_F(4, 26)
  return 0;
}
