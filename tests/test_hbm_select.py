"""Agent selection of the in-task HBM counter tool (``native/th_hbm_select.h``), compiled with the
host compiler alone: a task reserved GPU 3 through HIP_VISIBLE_DEVICES must count GPU 3, not GPU 0."""
import shutil
import subprocess
from pathlib import Path

import pytest

HDR = Path(__file__).resolve().parents[1] / "tensorhive_fixed_amd" / "native"

DRIVER = r"""
#include <stdio.h>
#include "th_hbm_select.h"
static const char* arg(const char* s) { return s[0] == '-' ? nullptr : s; }
int main(int argc, char** argv) {  // n hip_visible|- local_rank|- all
  auto v = th_hbm::select_agents(atoi(argv[1]), arg(argv[2]), arg(argv[3]), argv[4][0] == '1');
  for (size_t i = 0; i < v.size(); ++i) printf("%s%d", i ? "," : "", v[i]);
  printf("\n");
  return 0;
}
"""


@pytest.fixture(scope="module")
def select(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    d = tmp_path_factory.mktemp("hbmsel")
    (d / "drv.cpp").write_text(DRIVER)
    subprocess.run([cxx, "-std=c++17", "-O1", f"-I{HDR}", str(d / "drv.cpp"), "-o", str(d / "drv")], check=True)

    def run(n, vis, rank, all_agents=False):
        out = subprocess.run([str(d / "drv"), str(n), vis or "-", rank or "-", "1" if all_agents else "0"],
                             capture_output=True, text=True, check=True).stdout.strip()
        return [int(x) for x in out.split(",")] if out else []
    return run


def test_unrestricted_task_counts_every_gpu(select):
    assert select(8, None, None) == list(range(8))


def test_reserved_gpus_follow_hip_visible_devices(select):
    assert select(8, "3", None) == [3]
    assert select(8, "5,2", None) == [5, 2]
    assert select(8, "3", "0") == [3]  # torchrun rank 0 of a job reserved GPU 3
    assert select(8, "4,5,6,7", "2") == [6]
    assert select(8, "4,5,6,7", "2", all_agents=True) == [4, 5, 6, 7]


def test_plain_rank_without_visibility_and_odd_inputs(select):
    assert select(8, None, "5") == [5]
    assert select(8, "1,9", None) == [1]  # out-of-range entries dropped
    assert select(8, "GPU-1234abcd", "1") == [1]  # UUIDs cannot be mapped here: no filter
    assert select(2, "7", "0") == []  # nothing visible: nothing sampled
