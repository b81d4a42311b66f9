"""The C-ABI boundary (include/neus2_hip.h): the library loads without a GPU, exports every declared
symbol, and the ctypes mirrors in neus2_amd/_lib.py have the C struct layouts (checked against gcc
compiling the header). No compute is called here."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "neus2_hip.h")


def declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*|void|uint32_t)\s+(neus_\w+)\s*\(", text, flags=re.M)))


def test_exports_list_matches_header():
    from neus2_amd._lib import EXPORTS
    assert sorted(EXPORTS) == declared()


def test_library_loads_and_exports_every_symbol():
    from neus2_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libneus2_hip.so not built (run __graft_entry__.build())")
    lib = C.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared() if not hasattr(lib, s)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(l.split()[-1] for l in out.splitlines() if " T " in l)
    assert set(declared()) <= exported


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    """No fallback path: a missing .so raises instead of silently computing elsewhere."""
    from neus2_amd import _lib
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(RuntimeError):
        _lib.lib()


PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "neus2_hip.h"
#define S(T) printf(#T " %zu\n", sizeof(T));
#define O(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
int main(void) {
  S(NeusNetworkConfig) S(NeusImage) S(NeusTrainStats) S(NeusNetLayout) S(NeusDataParallelInfo) S(NeusTrainingOptions)
  O(NeusTrainingOptions, depth_supervision_lambda)
  O(NeusNetworkConfig, fixed_rays_per_batch) O(NeusNetworkConfig, seed) O(NeusNetworkConfig, batch_size)
  O(NeusImage, rgba8) O(NeusImage, xform)
  O(NeusTrainStats, ray_loss) O(NeusTrainStats, n_rays_with_samples) O(NeusTrainStats, trained_samples_total)
  O(NeusNetLayout, per_level_scale) O(NeusNetLayout, n_levels)
  O(NeusTrainStats, pre_samples_total) O(NeusTrainStats, occ_updates) O(NeusTrainStats, evaluated_samples_total)
  O(NeusTrainStats, evaluated_samples_last)
  O(NeusDataParallelInfo, collective_calls) O(NeusDataParallelInfo, last_step_allreduce_bytes)
  printf("NEUS_N_PHASES %d\n", NEUS_N_PHASES);
  return 0;
}
"""


def test_struct_layouts_match_header(tmp_path):
    from neus2_amd import _lib
    src = tmp_path / "probe.c"
    src.write_text(PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    vals = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines())
    for name in ("NeusNetworkConfig", "NeusImage", "NeusTrainStats", "NeusNetLayout", "NeusDataParallelInfo", "NeusTrainingOptions"):
        T = getattr(_lib, name)
        assert C.sizeof(T) == int(vals[name]), name
        for key, v in vals.items():
            if key.startswith(name + "."):
                assert getattr(T, key.split(".")[1]).offset == int(v), key
    from neus2_amd.pyngp import PHASES
    assert len(PHASES) == int(vals["NEUS_N_PHASES"])


def test_mc_table_matches_oracle_restatement():
    """neus_mc_table (host-only entry point: the generated case table the kernels upload) equals the
    oracle's independent restatement (oracle/mc_table.py)."""
    import ctypes as C
    import sys
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import mc_table
    from neus2_amd._lib import check, lib
    out = np.zeros((256, 19), np.int8)
    check(lib().neus_mc_table(C.c_void_p(out.ctypes.data)))
    np.testing.assert_array_equal(out, mc_table.build_table())


@pytest.mark.parametrize("n_in,n_out,net,msg", [
    (32, 3, '{"otype": "FullyFusedMLP", "n_neurons": 48, "n_hidden_layers": 2}', "only supports 16, 32, 64, and 128 neurons"),
    (32, 3, '{"otype": "FullyFusedMLP", "n_neurons": 64, "n_hidden_layers": 0}', "at least 1 hidden layer"),
    (32, 3, '{"otype": "FullyFusedMLP", "n_neurons": 64, "activation": "Sine"}', "Sine has no backward"),
    (32, 3, '{"otype": "CutlassResNet"}', "only FullyFusedMLP"),
    (0, 3, '{"otype": "FullyFusedMLP"}', "input dims"),
])
def test_create_network_validates_config(n_in, n_out, net, msg):
    """tcnn create_network's FullyFusedMLP checks (fully_fused_mlp.cu:816-879, network.cu:111-120) run before any device
    call: a bad config is an error status with tcnn's message (no GPU needed)."""
    from neus2_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libneus2_hip.so not built")
    lib = _lib.lib()
    h = C.c_void_p()
    rc = lib.neus_module_create_network(C.c_uint32(n_in), C.c_uint32(n_out), net.encode(), C.c_uint32(1024), C.byref(h))
    assert rc != 0 and msg in lib.neus_last_error().decode()
