"""rt_acos (tinyraytracerinrust_amd/csrc/rt_math.h), the acos the render kernels use, compiled
for the host with the same no-contraction flags and checked against glibc's acos -- the libm the
reference's Rust `f64::acos` calls (vector.rs:69-71 angle, sphere.rs:82-114 UV).  The device build
is the same source; the GPU parity tests cover it end to end."""
import pathlib
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
HARNESS = r"""
#include "rt_math.h"
#include <cstdio>
#include <cstring>
#include <cstdint>
#include <cmath>
#include <random>
int main() {
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  long n = 2000000, diff = 0, worst = 0;
  for (long i = 0; i < n; ++i) {
    double x = u(rng);
    if (i % 3 == 1) x *= 1e-3;                                   // near pi/2
    if (i % 7 == 2) x = (x > 0 ? 1 : -1) * (1.0 - std::fabs(x) * 1e-6);   // near 0 and pi
    double a = rt_acos(x), b = std::acos(x);
    if (a != b) { int64_t ia, ib; memcpy(&ia, &a, 8); memcpy(&ib, &b, 8);
                  long d = ia > ib ? ia - ib : ib - ia; ++diff; if (d > worst) worst = d; }
  }
  const double sp[] = {1.0, -1.0, 0.0, -0.0, 0.5, -0.5, 0x1p-60, -0x1p-60, 1e-300};
  int bad = 0;
  for (double x : sp) bad += rt_acos(x) != std::acos(x);
  bad += !std::isnan(rt_acos(NAN)) + !std::isnan(rt_acos(1.5)) + !std::isnan(rt_acos(-2.0));
  printf("%ld %ld %ld %d\n", n, diff, worst, bad);
}
"""


def test_rt_acos_matches_glibc(tmp_path):
    src = tmp_path / "h.cpp"
    src.write_text(HARNESS)
    exe = tmp_path / "h"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-mfma", "-std=c++17",
                    f"-I{ROOT / 'tinyraytracerinrust_amd' / 'csrc'}", str(src), "-o", str(exe), "-lm"],
                   check=True)
    n, diff, worst, bad = map(int, subprocess.run([str(exe)], check=True, capture_output=True,
                                                  text=True).stdout.split())
    print(f"rt_acos vs glibc: {diff}/{n} differ, max {worst} ulp, special-value mismatches {bad}")
    assert bad == 0
    assert worst <= 1
    assert diff / n < 0.01        # ocml's acos: ~6.5 % (profiles/r01_libm_probe.txt)


CR_HARNESS = r"""
#include "rt_math.h"
#include <quadmath.h>
#include <cmath>
#include <cstdio>
#include <random>
int main() {
  std::mt19937_64 rng(11);
  std::uniform_real_distribution<double> u(-1.0, 1.0), up(0.0, 3.141592653589793);
  long n = 600000, ma = 0, ms = 0, ga = 0, gs = 0, ca = 0, cs = 0;
  for (long i = 0; i < n; ++i) {
    double x = u(rng);
    if (i % 5 == 1) x = (x > 0 ? 1 : -1) * (1.0 - std::fabs(x) * 1e-9);      // near +-1
    if (i % 5 == 2) x *= 1e-4;                                                 // near 0
    if (i % 5 == 3) x = (x > 0 ? 1 : -1) * (0.5 + x * 1e-6);                   // the branch point
    const double c = (double)acosq((__float128)x), a = rt_acos_cr(x), g = std::acos(x);
    ma += a != c; ga += g != c; ca += a != g;
    double p = up(rng);
    if (i % 4 == 1) p = 3.141592653589793 - p * 1e-7;                           // near pi
    if (i % 4 == 2) p = 0.7853981633974483 + (p - 1.5) * 1e-9;                 // pi/4
    if (i % 4 == 3) p = 1.5707963267948966 + (p - 1.5) * 1e-7;                 // pi/2
    if (p < 0) p = -p;
    const double cs_ = (double)sinq((__float128)p), s = rt_sin_cr(p), gs_ = std::sin(p);
    ms += s != cs_; gs += gs_ != cs_; cs += s != gs_;
  }
  const double sp[] = {1.0, -1.0, 0.0, -0.0, 0.5, -0.5, 0x1p-60, 1e-300};
  int bad = 0;
  for (double x : sp) bad += rt_acos_cr(x) != (double)acosq((__float128)x);
  bad += !std::isnan(rt_acos_cr(NAN)) + !std::isnan(rt_acos_cr(1.5));
  bad += rt_sin_cr(0.0) != 0.0 || rt_sin_cr(0x1.921fb54442d18p+1) != std::sin(0x1.921fb54442d18p+1);
  printf("%ld %ld %ld %ld %ld %ld %ld %d\n", n, ma, ga, ca, ms, gs, cs, bad);
}
"""


def test_correctly_rounded_acos_sin(tmp_path):
    """rt_acos_cr / rt_sin_cr (rt_math.h: double-double evaluation, one rounding), the sphere UV's
    texel-boundary path: correctly rounded -- equal to libquadmath's 113-bit acosq / sinq rounded to
    double -- on every sampled input, and therefore equal to glibc's acos / sin wherever glibc is
    correctly rounded (it is not on ~0.05 % / ~0.14 % of inputs; the printed counts say how often)."""
    import shutil
    if not shutil.which("g++"):
        pytest.skip("no g++")
    src = tmp_path / "cr.cpp"
    src.write_text(CR_HARNESS)
    exe = tmp_path / "cr"
    r = subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17",
                        f"-I{ROOT / 'tinyraytracerinrust_amd' / 'csrc'}", str(src), "-o", str(exe), "-lquadmath", "-lm"],
                       capture_output=True, text=True)
    if r.returncode != 0 and "quadmath" in r.stderr:
        pytest.skip("libquadmath not available")
    assert r.returncode == 0, r.stderr[-2000:]
    n, ma, ga, ca, ms, gs, cs, bad = map(int, subprocess.run([str(exe)], check=True, capture_output=True,
                                                             text=True).stdout.split())
    print(f"acos_cr != CR {ma}/{n} (glibc != CR {ga}, acos_cr != glibc {ca}); "
          f"sin_cr != CR {ms}/{n} (glibc != CR {gs}, sin_cr != glibc {cs}); special {bad}")
    assert ma == 0 and ms == 0 and bad == 0
    assert ca == ga and cs == gs          # every disagreement with glibc is one of glibc's own roundings
