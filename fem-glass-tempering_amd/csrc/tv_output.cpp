// Time-series output of the state fields: XDMF 3 (XML) over raw little-endian
// binary, written by a host thread while the device runs the next step.
//
// Replaces the reference's output subsystem (ThermoViscoProblem.py:246-276
// _write_initial_output, :357-364 _write_output, :614-620 _finalize): VTX/BP4
// files for T, phi, Tf and xi and an XDMF/HDF5 file for sigma, written every
// step through dolfinx.io (ADIOS2 / HDF5, which are not available here).  The
// same five fields are written, one XDMF series per field (<name>.xdmf next to
// <name>.bin); ParaView and meshio read them.
//
// Device -> host path (tv_output_write): on the context's compute stream the
// fields are gathered into a device staging area in the reference's interleaved
// layout (k_interleave); an event hands it to a separate copy stream, which
// copies it into one of two pinned host buffer sets; a writer thread waits for
// the copy, appends the arrays to the .bin files and rewrites the .xdmf index.
// tv_output_write returns as soon as the copies are queued, so the next time
// step's Newton solve overlaps the PCIe copy and the file writes; it blocks
// only while both buffer sets are still in flight (back-pressure).
//
// The file format layer (XdmfSeries) has no HIP dependency and is reachable
// without a GPU through tv_xdmf_* (tests/test_output.py round-trips it on CPU).
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include <algorithm>

#include "tv_internal.h"

namespace tv {

// ---- file format ---------------------------------------------------------------
struct XdmfField {
  std::string name;
  int ncomp = 1;          // values per node (1, d*d)
  bool cell_nodes = false;  // DG: on the discontinuous copy of the mesh
  FILE* bin = nullptr;
  std::vector<std::pair<double, long long>> steps;  // (time, byte offset)
};

struct XdmfSeries {
  std::string dir;
  int dim = 1;
  int64_t n_nodes = 0, n_cells = 0, n_dnodes = 0;  // continuous / discontinuous node counts
  std::vector<XdmfField> fields;
  std::string err;

  static const char* topo_type(int d) { return d == 1 ? "Polyline" : (d == 2 ? "Quadrilateral" : "Hexahedron"); }
  static const char* attr_type(int ncomp) { return ncomp == 1 ? "Scalar" : (ncomp == 9 ? "Tensor" : "Matrix"); }

  // geometry (x, y, z per node) and cells (2^d node ids per cell, VTK order)
  bool write_mesh(const char* prefix, const std::vector<double>& xyz, const std::vector<int64_t>& cells) {
    const std::string g = dir + "/" + prefix + "_geometry.bin", t = dir + "/" + prefix + "_topology.bin";
    FILE* f = std::fopen(g.c_str(), "wb");
    if (!f) return fail("cannot write " + g);
    std::fwrite(xyz.data(), sizeof(double), xyz.size(), f);
    std::fclose(f);
    f = std::fopen(t.c_str(), "wb");
    if (!f) return fail("cannot write " + t);
    std::fwrite(cells.data(), sizeof(int64_t), cells.size(), f);
    std::fclose(f);
    return true;
  }

  bool fail(const std::string& m) {
    err = m;
    return false;
  }

  // the discontinuous copy of the mesh, written when the first DG field opens
  std::vector<double> dg_xyz;
  std::vector<int64_t> dg_cells;
  bool dg_written = false;

  bool open_field(const std::string& name, int ncomp, bool cell_nodes) {
    if (cell_nodes && !dg_written) {
      if (!write_mesh("mesh_dg", dg_xyz, dg_cells)) return false;
      dg_written = true;
      std::vector<double>().swap(dg_xyz);
      std::vector<int64_t>().swap(dg_cells);
    }
    XdmfField fl;
    fl.name = name;
    fl.ncomp = ncomp;
    fl.cell_nodes = cell_nodes;
    const std::string b = dir + "/" + name + ".bin";
    fl.bin = std::fopen(b.c_str(), "wb");
    if (!fl.bin) return fail("cannot write " + b);
    fields.push_back(std::move(fl));
    return rewrite_index(fields.back());
  }

  bool append(size_t k, double t, const double* v, size_t n) {
    std::string e;
    if (!append_field(k, t, v, n, e)) return fail(e);
    return true;
  }
  // touches field k's file and index only (fields are written concurrently)
  bool append_field(size_t k, double t, const double* v, size_t n, std::string& e) {
    XdmfField& fl = fields[k];
    const long long off = (long long)std::ftell(fl.bin);
    if (std::fwrite(v, sizeof(double), n, fl.bin) != n) {
      e = "short write of " + fl.name + ".bin";
      return false;
    }
    std::fflush(fl.bin);
    fl.steps.emplace_back(t, off);
    return rewrite_index(fl, &e);
  }

  // the whole index is rewritten at every step, so the .xdmf file is valid
  // XML at any moment (a run stopped half-way leaves a readable series)
  bool rewrite_index(const XdmfField& fl, std::string* e = nullptr) {
    const std::string path = dir + "/" + fl.name + ".xdmf", tmp = path + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "w");
    if (!f) {
      if (e) *e = "cannot write " + tmp;
      return e ? false : fail("cannot write " + tmp);
    }
    const char* pre = fl.cell_nodes ? "mesh_dg" : "mesh";
    const int64_t nn = fl.cell_nodes ? n_dnodes : n_nodes;
    const int npc = 1 << dim;
    std::fprintf(f, "<?xml version=\"1.0\"?>\n<Xdmf Version=\"3.0\">\n <Domain>\n");
    std::fprintf(f, "  <Grid Name=\"%s\" GridType=\"Collection\" CollectionType=\"Temporal\">\n", fl.name.c_str());
    for (const auto& st : fl.steps) {
      std::fprintf(f, "   <Grid Name=\"%s\" GridType=\"Uniform\">\n    <Time Value=\"%.17g\"/>\n", fl.name.c_str(),
                   st.first);
      std::fprintf(f,
                   "    <Topology TopologyType=\"%s\" NumberOfElements=\"%lld\" NodesPerElement=\"%d\">\n"
                   "     <DataItem Format=\"Binary\" DataType=\"Int\" Precision=\"8\" Endian=\"Little\" "
                   "Dimensions=\"%lld %d\">%s_topology.bin</DataItem>\n    </Topology>\n",
                   topo_type(dim), (long long)n_cells, npc, (long long)n_cells, npc, pre);
      std::fprintf(f,
                   "    <Geometry GeometryType=\"XYZ\">\n"
                   "     <DataItem Format=\"Binary\" DataType=\"Float\" Precision=\"8\" Endian=\"Little\" "
                   "Dimensions=\"%lld 3\">%s_geometry.bin</DataItem>\n    </Geometry>\n",
                   (long long)nn, pre);
      std::fprintf(f,
                   "    <Attribute Name=\"%s\" AttributeType=\"%s\" Center=\"Node\">\n"
                   "     <DataItem Format=\"Binary\" DataType=\"Float\" Precision=\"8\" Endian=\"Little\" "
                   "Seek=\"%lld\" Dimensions=\"%lld %d\">%s.bin</DataItem>\n    </Attribute>\n   </Grid>\n",
                   fl.name.c_str(), attr_type(fl.ncomp), st.second, (long long)nn, fl.ncomp, fl.name.c_str());
    }
    std::fprintf(f, "  </Grid>\n </Domain>\n</Xdmf>\n");
    std::fclose(f);
    if (std::rename(tmp.c_str(), path.c_str()) != 0) {
      if (e) *e = "cannot rename " + tmp;
      return e ? false : fail("cannot rename " + tmp);
    }
    return true;
  }

  void close() {
    for (auto& fl : fields)
      if (fl.bin) {
        std::fclose(fl.bin);
        fl.bin = nullptr;
      }
  }
  ~XdmfSeries() { close(); }
};

// rectilinear mesh (per-axis coordinates, global numbering i + N0 (j + N1 k)):
// continuous nodes and cells, and the discontinuous copy (node = (cell, l))
// X[s]: node coordinates along storage axis s (s < 3; a single node for a
// degenerate axis), phys[s]: the physical axis of storage axis s (-1: none)
static void rect_mesh(int dim, const std::vector<std::vector<double>>& X, const int* phys, std::vector<double>& xyz,
                      std::vector<int64_t>& cells, std::vector<double>& dxyz, std::vector<int64_t>& dcells) {
  int N[3] = {1, 1, 1}, C[3] = {1, 1, 1};
  for (int a = 0; a < 3; ++a) {
    N[a] = (int)X[a].size();
    C[a] = std::max(1, N[a] - 1);
  }
  const int64_t nn = (int64_t)N[0] * N[1] * N[2], nc = (int64_t)C[0] * C[1] * C[2];
  xyz.assign(3 * nn, 0.0);
  for (int64_t v = 0; v < nn; ++v) {
    const int64_t c[3] = {v % N[0], (v / N[0]) % N[1], v / ((int64_t)N[0] * N[1])};
    for (int a = 0; a < 3; ++a)
      if (phys[a] >= 0) xyz[3 * v + phys[a]] = X[a][c[a]];
  }
  // VTK vertex order of the tensor cell (local l = a + 2 b + 4 c)
  static const int vtk[8] = {0, 1, 3, 2, 4, 5, 7, 6};
  const int npc = 1 << dim;
  cells.assign(npc * nc, 0);
  dcells.assign(npc * nc, 0);
  dxyz.assign(3 * npc * nc, 0.0);
  // local vertex bit k belongs to the k-th non-degenerate storage axis
  int bit_of[3] = {-1, -1, -1};
  for (int a = 0, k = 0; a < 3; ++a)
    if (N[a] > 1) bit_of[a] = k++;
  for (int64_t e = 0; e < nc; ++e) {
    const int64_t c[3] = {e % C[0], (e / C[0]) % C[1], e / ((int64_t)C[0] * C[1])};
    for (int q = 0; q < npc; ++q) {
      const int l = (dim == 1) ? q : vtk[q];
      int64_t v = 0, s = 1;
      for (int a = 0; a < 3; ++a) {
        const int b = bit_of[a] >= 0 ? (l >> bit_of[a]) & 1 : 0;
        v += (c[a] + b) * s;
        s *= N[a];
      }
      cells[npc * e + q] = v;
      // discontinuous copy: dof (cell e, local l) in the reference's cell-major order
      const int64_t dn = npc * e + l;
      dcells[npc * e + q] = dn;
      for (int a = 0; a < 3; ++a) dxyz[3 * dn + a] = xyz[3 * v + a];
    }
  }
}

}  // namespace tv

using namespace tv;

// ---- host-only format API (no GPU) ---------------------------------------------
struct tv_xdmf {
  XdmfSeries s;
};

extern "C" {

void* tv_xdmf_open(const char* dir, int dim, const int* n_cells, const double* const* coords) {
  if (!dir || dim < 1 || dim > 3 || !n_cells || !coords) return nullptr;
  auto* h = new tv_xdmf();
  h->s.dir = dir;
  h->s.dim = dim;
  std::vector<std::vector<double>> X(3, std::vector<double>(1, 0.0));
  int phys[3] = {-1, -1, -1};
  for (int a = 0; a < dim; ++a) {
    X[a].assign(coords[a], coords[a] + n_cells[a] + 1);
    phys[a] = a;
  }
  std::vector<double> xyz, dxyz;
  std::vector<int64_t> cells, dcells;
  rect_mesh(dim, X, phys, xyz, cells, dxyz, dcells);
  h->s.n_nodes = (int64_t)xyz.size() / 3;
  h->s.n_cells = (int64_t)cells.size() >> dim;
  h->s.n_dnodes = (int64_t)dxyz.size() / 3;
  if (!h->s.write_mesh("mesh", xyz, cells)) {
    delete h;
    return nullptr;
  }
  h->s.dg_xyz.swap(dxyz);
  h->s.dg_cells.swap(dcells);
  return h;
}

int tv_xdmf_add_field(void* xh, const char* name, int ncomp, int discontinuous) {
  auto* h = static_cast<tv_xdmf*>(xh);
  if (!h || !name || ncomp < 1) return TV_ERR_ARG;
  return h->s.open_field(name, ncomp, discontinuous != 0) ? TV_OK : TV_ERR_STATE;
}

int tv_xdmf_append(void* xh, int field, double t, const double* values, size_t n_values) {
  auto* h = static_cast<tv_xdmf*>(xh);
  if (!h || !values || field < 0 || field >= (int)h->s.fields.size()) return TV_ERR_ARG;
  const XdmfField& fl = h->s.fields[field];
  const int64_t nn = fl.cell_nodes ? h->s.n_dnodes : h->s.n_nodes;
  if ((int64_t)n_values != nn * fl.ncomp) return TV_ERR_ARG;
  return h->s.append(field, t, values, n_values) ? TV_OK : TV_ERR_STATE;
}

void tv_xdmf_close(void* xh) { delete static_cast<tv_xdmf*>(xh); }

}  // extern "C"

// ---- asynchronous device output -----------------------------------------------
namespace tv {

struct OutJob {
  int set;
  double t;
};

struct Output {
  XdmfSeries series;
  std::vector<size_t> field_n;    // values per field (owned dofs x bs)
  std::vector<size_t> field_off;  // offset in a staging set (doubles)
  size_t set_n = 0;
  double* dstage[2] = {nullptr, nullptr};
  double* hstage[2] = {nullptr, nullptr};
  hipEvent_t ready[2] = {nullptr, nullptr}, copied[2] = {nullptr, nullptr};
  hipStream_t copy = nullptr;
  bool busy[2] = {false, false};
  int next = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<OutJob> q;
  bool stop = false;
  std::string err;
  std::thread th;
  int device = 0;

  void run() {
    hipSetDevice(device);
    for (;;) {
      OutJob j;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || !q.empty(); });
        if (q.empty()) return;
        j = q.front();
        q.pop_front();
      }
      // a failed copy (device fault) must not append stale pinned data: the
      // error is recorded and this step's write skipped
      const hipError_t ce = hipEventSynchronize(copied[j.set]);
      std::vector<std::string> errs(field_n.size());
      if (ce != hipSuccess) {
        errs[0] = std::string("output: device-to-host copy failed: ") + hipGetErrorString(ce);
      } else {
        // one thread per field: the page-cache copy of one fwrite is single-threaded
        std::vector<std::thread> ws;
        for (size_t k = 0; k < field_n.size(); ++k)
          ws.emplace_back([&, k] {
            if (!series.append_field(k, j.t, hstage[j.set] + field_off[k], field_n[k], errs[k])) return;
          });
        for (auto& w : ws) w.join();
      }
      for (const auto& e : errs)
        if (!e.empty()) {
          std::lock_guard<std::mutex> lk(mu);
          if (err.empty()) err = e;
        }
      {
        std::lock_guard<std::mutex> lk(mu);
        busy[j.set] = false;
      }
      cv.notify_all();
    }
  }
};

Output* output_create(const std::string& dir, int dim, const std::vector<std::vector<double>>& Xs, const int* phys,
                      std::string& err) {
  auto* o = new Output();
  o->series.dir = dir;
  o->series.dim = dim;
  std::vector<double> xyz, dxyz;
  std::vector<int64_t> cells, dcells;
  rect_mesh(dim, Xs, phys, xyz, cells, dxyz, dcells);
  o->series.n_nodes = (int64_t)xyz.size() / 3;
  o->series.n_cells = (int64_t)cells.size() >> dim;
  o->series.n_dnodes = (int64_t)dxyz.size() / 3;
  if (!o->series.write_mesh("mesh", xyz, cells)) {
    err = o->series.err;
    delete o;
    return nullptr;
  }
  o->series.dg_xyz.swap(dxyz);
  o->series.dg_cells.swap(dcells);
  return o;
}

// unstructured mesh: vertices (3 per vertex) and cells (2^dim per cell, tensor
// order) as given; cells written in VTK vertex order
Output* output_create_unstructured(const std::string& dir, int dim, const std::vector<double>& xyz,
                                   const std::vector<int64_t>& cells, std::string& err) {
  auto* o = new Output();
  o->series.dir = dir;
  o->series.dim = dim;
  static const int vtk[8] = {0, 1, 3, 2, 4, 5, 7, 6};
  const int npc = 1 << dim;
  std::vector<int64_t> vc(cells.size());
  for (size_t e = 0; e < cells.size() / npc; ++e)
    for (int q = 0; q < npc; ++q) vc[e * npc + q] = cells[e * npc + vtk[q]];
  o->series.n_nodes = (int64_t)xyz.size() / 3;
  o->series.n_cells = (int64_t)(cells.size() / npc);
  o->series.n_dnodes = 0;
  if (!o->series.write_mesh("mesh", xyz, vc)) {
    err = o->series.err;
    delete o;
    return nullptr;
  }
  return o;
}

bool output_add_field(Output* o, const std::string& name, int ncomp, bool dg, size_t n_values, std::string& err) {
  if (!o->series.open_field(name, ncomp, dg)) {
    err = o->series.err;
    return false;
  }
  o->field_n.push_back(n_values);
  o->field_off.push_back(o->set_n);
  o->set_n += n_values;
  return true;
}

bool output_start(Output* o, int device, std::string& err) {
  o->device = device;
  for (int k = 0; k < 2; ++k) {
    if (hipMalloc(&o->dstage[k], sizeof(double) * std::max<size_t>(1, o->set_n)) != hipSuccess ||
        hipHostMalloc(&o->hstage[k], sizeof(double) * std::max<size_t>(1, o->set_n)) != hipSuccess ||
        hipEventCreateWithFlags(&o->ready[k], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&o->copied[k], hipEventDisableTiming) != hipSuccess) {
      err = "output: device / pinned staging allocation failed";
      return false;
    }
  }
  if (hipStreamCreateWithFlags(&o->copy, hipStreamNonBlocking) != hipSuccess) {
    err = "output: copy stream creation failed";
    return false;
  }
  o->th = std::thread([o] { o->run(); });
  return true;
}

// staging set for the next write (waits while both are in flight); its device
// area and the per-field offsets
double* output_acquire(Output* o, int* set) {
  std::unique_lock<std::mutex> lk(o->mu);
  o->cv.wait(lk, [&] { return !o->busy[o->next]; });
  *set = o->next;
  o->busy[o->next] = true;
  o->next ^= 1;
  return o->dstage[*set];
}
size_t output_offset(const Output* o, size_t k) { return o->field_off[k]; }

// gives an acquired set back without a write (its submission failed), so a
// later output_acquire does not wait for it forever
void output_release(Output* o, int set) {
  {
    std::lock_guard<std::mutex> lk(o->mu);
    o->busy[set] = false;
  }
  o->cv.notify_all();
}

// the gathers into set `set` are queued on `compute`: copy after them on the
// copy stream, then hand the set to the writer thread
bool output_submit(Output* o, int set, double t, hipStream_t compute, std::string& err) {
  if (hipEventRecord(o->ready[set], compute) != hipSuccess || hipStreamWaitEvent(o->copy, o->ready[set], 0) != hipSuccess ||
      hipMemcpyAsync(o->hstage[set], o->dstage[set], sizeof(double) * o->set_n, hipMemcpyDeviceToHost, o->copy) !=
          hipSuccess ||
      hipEventRecord(o->copied[set], o->copy) != hipSuccess) {
    err = "output: copy submission failed";
    output_release(o, set);
    return false;
  }
  {
    std::lock_guard<std::mutex> lk(o->mu);
    o->q.push_back({set, t});
    if (!o->err.empty()) err = o->err;
  }
  o->cv.notify_all();
  return err.empty();
}

// drains the queue and frees everything; returns the writer's first error
std::string output_destroy(Output* o) {
  {
    std::lock_guard<std::mutex> lk(o->mu);
    o->stop = true;
  }
  o->cv.notify_all();
  if (o->th.joinable()) o->th.join();
  std::string e = o->err;
  for (int k = 0; k < 2; ++k) {
    if (o->dstage[k]) hipFree(o->dstage[k]);
    if (o->hstage[k]) hipHostFree(o->hstage[k]);
    if (o->ready[k]) hipEventDestroy(o->ready[k]);
    if (o->copied[k]) hipEventDestroy(o->copied[k]);
  }
  if (o->copy) hipStreamDestroy(o->copy);
  o->series.close();
  delete o;
  return e;
}

}  // namespace tv
