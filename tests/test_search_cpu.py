"""The device lower-bound searches (kernels.hip: lower_bound, lower_bound_interp,
lower_bound_back, lower_bound_near) compiled for the host with gcc and checked against a linear
scan on random sorted series: regular, jittered, duplicated and gapped
timestamps, every sub-range shape.  They decide where a query's span starts
(k_prep's seek, which stands for Span.java:360 seekRow and 464 seek) and where each fold
window starts (k_fold_prep), so any disagreement is a parity bug."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "opentsdb_amd", "csrc", "kernels.hip")

HARNESS = r"""
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#define DEV static
%s
static int64_t ref(const int64_t* ts, int64_t a, int64_t b, int64_t t) {
  while (a < b && ts[a] < t) a++;
  return a;
}
int main(void) {
  static int64_t ts[400];
  long bad = 0, n = 0;
  srand(7);
  for (int it = 0; it < 20000; it++) {
    const int len = rand() %% 300, mode = rand() %% 4;
    int64_t v = rand() %% 5;
    for (int i = 0; i < len; i++) {
      v += mode == 0 ? 10 : mode == 1 ? rand() %% 3
         : mode == 2 ? (rand() %% 50 == 0 ? 100000 : rand() %% 20) : 0;
      ts[i] = v;
    }
    for (int q = 0; q < 40; q++) {
      const int a = len ? rand() %% (len + 1) : 0;
      const int b = a + (len - a ? rand() %% (len - a + 1) : 0);
      const int64_t t = (len ? ts[rand() %% len] : 0) + rand() %% 5 - 2;
      const int64_t r = ref(ts, a, b, t);
      n++;
      bad += lower_bound(ts, a, b, t) != r;
      bad += lower_bound_interp(ts, a, b, t) != r;
      bad += lower_bound_back(ts, a, b, t) != r;
      bad += lower_bound_near(ts, a, b, t) != r;
    }
  }
  printf("%%ld %%ld\n", n, bad);
  return bad != 0;
}
"""


def _function(text, name):
    m = re.search(r"^DEV int64_t %s\(.*?^}\n" % name, text, re.S | re.M)
    assert m, name
    return m.group(0)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc absent")
def test_lower_bounds_match_linear_scan(tmp_path):
    text = open(SRC).read()
    body = "".join(_function(text, n) for n in
                   ("lower_bound", "lower_bound_interp", "lower_bound_back",
                    "lower_bound_near"))
    c = tmp_path / "lb.c"
    c.write_text(HARNESS % body)
    exe = tmp_path / "lb"
    subprocess.run(["gcc", "-O2", "-o", str(exe), str(c)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    n, bad = map(int, out.stdout.split())
    assert n == 800000 and bad == 0, out.stdout

