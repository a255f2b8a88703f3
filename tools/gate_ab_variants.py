"""Build tools/gate_ab.hip against ablated copies of csrc/gemm_half.hip's
GATE epilogue (scratch copies under /tmp/gate_ab/<variant>/pkg/csrc): full, rg stores
only, no xc / z loads, no wait for the previous row tile, no gate math."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "datamining_recblr_amd", "csrc")


def variant(name, s):
    if name == "full":
        return s
    if name == "rgonly":
        a = s.index("#pragma unroll 1\n      for (int q = 0; q < NCH; ++q) {")
        b = s.index("      }\n    }\n  };\n\n  bool stored_prev") + len("      }\n")
        return s[:a] + s[b:]
    if name == "noload":
        s = s.replace("xv[j] = o < lim ? xw[xo + o * ldx] : 0.0f;", "xv[j] = 0.5f + o;")
        return s.replace("zv[j] = o < lim ? zw[zo + o * zrs] : 0.0f;", "zv[j] = 0.25f * o;")
    if name == "nowait":
        return s.replace("const bool need = mt_g > 0 && (tinfo & 255) != 0;",
                         "const bool need = false && tinfo;")
    if name == "nomath":
        old = """            const float a = fexp(nsp * fsigm(acc[0][j] + br));
            const float beta = fsqrt(1.0f - a * a + 1e-8f) * fsigm(acc[NCH][j] + bi);"""
        assert old in s
        return s.replace(old, """            const float a = acc[0][j] * nsp + br;
            const float beta = acc[NCH][j] + bi;""")
    raise ValueError(name)


def main(names):
    src = open(os.path.join(SRC, "gemm_half.hip")).read()
    for n in names:
        top = f"/tmp/gate_ab/{n}"
        d = os.path.join(top, "pkg", "csrc")   # common.h includes ../../include/
        shutil.rmtree(top, ignore_errors=True)
        shutil.copytree(SRC, d)
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(top, "include"))
        v = variant(n, src)
        assert n == "full" or v != src, n
        open(os.path.join(d, "gemm_half.hip"), "w").write(v)
        out = os.path.join(ROOT, "tools", "bin", f"gate_ab_{n}")
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-ffp-contract=off",
               "-std=c++17", "-I", os.path.join(ROOT, "include"), "-I", d, f"-DGEMM_DIR={d}",
               f"-DVARIANT={n}", os.path.join(ROOT, "tools", "gate_ab.hip"), "-o", out]
        subprocess.run(cmd, check=True)
        print("built", out)


if __name__ == "__main__":
    main(sys.argv[1:] or ["full", "rgonly", "noload", "nowait", "nomath"])
