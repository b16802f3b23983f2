"""Build a workgroup-timeline variant of libtvfem.so (timing build, not for
results): every k_cg_march workgroup records its start / end clock
(s_memrealtime, 100 MHz), its XCC id and its kind (0 plain tile, 1 face-chunk
tile with the march-axis facet prologue, 2 face workgroup) from lane 0 with
vector stores into a device buffer that tools/wgtrace/run.py reads back after
the last launch.  The sources are patched in a scratch copy; the tree is not
touched.

    python tools/wgtrace/build.py        # -> fem-glass-tempering_amd/tvfem/libtvfem_wgt.so
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
W = "/tmp/tvfem_var_wgt"


def patch(src):
    def rep(old, new, count=1):
        nonlocal src
        assert src.count(old) >= count, old
        src = src.replace(old, new, count)
    rep("namespace tv {\nnamespace {", """namespace tv {
__device__ unsigned long long tv_wgt_buf[4][16384];
struct WgtRec {
  unsigned long long t0;
  int b, k;
  __device__ ~WgtRec() {
    if (threadIdx.x == 0 && b < 16384) {
      tv_wgt_buf[0][b] = t0;
      tv_wgt_buf[1][b] = __builtin_amdgcn_s_memrealtime();
      tv_wgt_buf[2][b] = (unsigned long long)__builtin_amdgcn_s_getreg((15 << 11) | 20);
      tv_wgt_buf[3][b] = (unsigned long long)k;
    }
  }
};
namespace {""")
    # the first stamp_start(rt) is k_cg_march's
    rep("  static_assert(!POST || (MODE == MODE_JAC && !FUSEP), \"POST: plain Jacobian march only\");\n  stamp_start(rt);",
        "  static_assert(!POST || (MODE == MODE_JAC && !FUSEP), \"POST: plain Jacobian march only\");\n  stamp_start(rt);\n"
        "  WgtRec wgt_rec{__builtin_amdgcn_s_memrealtime(), (int)blockIdx.x, 0};")
    rep("  if (fidx >= 0) {\n    double ratio = 0.0;", "  if (fidx >= 0) {\n    wgt_rec.k = 2;\n    double ratio = 0.0;")
    rep("  const bool fq1 = (MODE == MODE_JAC) && q1 == nQ && bq_hi;",
        "  const bool fq1 = (MODE == MODE_JAC) && q1 == nQ && bq_hi;\n  wgt_rec.k = (fq0 || fq1) ? 1 : 0;")
    src += """
extern "C" int tv_wgt_read(unsigned long long* h) {
  return hipMemcpyFromSymbol(h, HIP_SYMBOL(tv::tv_wgt_buf), sizeof(unsigned long long) * 4 * 16384) == hipSuccess ? 0 : 1;
}
"""
    return src


def main():
    shutil.rmtree(W, ignore_errors=True)
    os.makedirs(W + "/tvfem")
    pk = os.path.join(ROOT, "fem-glass-tempering_amd")
    shutil.copytree(os.path.join(pk, "csrc"), W + "/csrc")
    shutil.copy(os.path.join(pk, "Makefile"), W + "/Makefile")
    mk = open(W + "/Makefile").read()
    mk = mk.replace("-I../include", "-I" + os.path.join(ROOT, "include")).replace(
        "../include/tvfem.h", os.path.join(ROOT, "include", "tvfem.h"))
    open(W + "/Makefile", "w").write(mk)
    p = W + "/csrc/tv_cg.hip"
    src = patch(open(p).read())
    open(p, "w").write(src)
    subprocess.run(["make", "-j8"], cwd=W, check=True, stdout=subprocess.DEVNULL)
    shutil.copy(W + "/tvfem/libtvfem.so", os.path.join(pk, "tvfem", "libtvfem_wgt.so"))
    print("built libtvfem_wgt.so")


if __name__ == "__main__":
    sys.exit(main())
