"""Regression guard on the gfx950 code objects inside librsc.so (no GPU needed): the latency-bound
kernels of the hot path must run without scratch (private segment) — a stack round trip inside a
dependent FP64 chain costs microseconds (DESIGN §9 scratch audit: the Refine's out-of-line
`wave_ordered_sum` and SearchByBoW's staged uint4 arrays were such cases).  Reads the AMDGPU
metadata notes with llvm-objdump / llvm-readelf from /opt/rocm; skipped when they are absent."""
import os
import shutil
import subprocess
import tempfile

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "orb-slam2-optimized_amd", "lib", "librsc.so")
LLVM = "/opt/rocm/lib/llvm/bin"

# kernels (demangled-name fragments) that must stay scratch-free
SCRATCH_FREE = [
    "pnp_eig_group_kernelILi4E", "pnp_eig_group_kernelILi5E", "pnp_eig_group_kernelILi6E",
    "pnp_betas_kernelILi4E", "pnp_scan_kernelILi8E", "pnp_refine_kernel",
    "sim3_solve_kernel", "sim3_scan_kernelILi4E", "sim3_pick_kernel",
    "sim3opt_kernel", "bow_topk_kernelILb0E", "bow_topk_kernelILb1E", "bow_walk_kernel",
    "sim3_search_kernel", "poseopt_kernel",
    "mlpnp_quad_kernelILi6ENS_7MlNoCov", "mlpnp_quad_kernelILi6ENS_12MlIndexedCov",
    # round 4: the NS = 7 / 8 variants too (their phase-1 state is parked as it is produced)
    "mlpnp_quad_kernelILi7ENS_7MlNoCov", "mlpnp_quad_kernelILi7ENS_12MlIndexedCov",
    "mlpnp_quad_kernelILi8ENS_7MlNoCov", "mlpnp_quad_kernelILi8ENS_12MlIndexedCov",
    # round 4: the rows form of the eigen stage for small launches (RSC_EIG_ROWS A/B variant)
    "pnp_eig_rows_kernelILi4E", "pnp_eig_rows_kernelILi5E", "pnp_eig_rows_kernelILi6E",
]


def _kernels():
    if not os.path.exists(LIB):
        pytest.skip("librsc.so not built")
    objdump, readelf = os.path.join(LLVM, "llvm-objdump"), os.path.join(LLVM, "llvm-readelf")
    if not (os.path.exists(objdump) and os.path.exists(readelf)):
        pytest.skip("llvm tools not available")
    out = {}
    with tempfile.TemporaryDirectory() as d:
        lib = os.path.join(d, "librsc.so")
        shutil.copy(LIB, lib)
        subprocess.run([objdump, "--offloading", lib], cwd=d, check=True, capture_output=True)
        cos = [f for f in os.listdir(d) if "gfx950" in f]
        assert cos, "no gfx950 code object in librsc.so"
        for f in cos:
            txt = subprocess.run([readelf, "--notes", os.path.join(d, f)], check=True, capture_output=True,
                                 text=True).stdout
            i = txt.index("---")
            j = txt.find("\n...", i)
            doc = yaml.safe_load(txt[i:j if j > 0 else len(txt)].replace("---", "", 1))
            for k in doc["amdhsa.kernels"]:
                out[k[".name"]] = k
    return out


# kernels whose VGPR spills go to AGPRs (v_accvgpr moves, no memory traffic): sim3opt_kernel holds
# the numeric Jacobian of an edge (14 perturbed-estimate errors in flight) beside the LM state, and
# the covariance variant of the MLPnP quad kernel the 6x6 bearing weights beside the 12x12 SVD, above
# the 256 architectural VGPRs of a wave; since round 4 both MLPnP NS = 6 variants evaluate the
# reference's generated Jacobian (mlpnpJacs, ~200 temporaries per correspondence, rsc_mlpnp_jac.h);
# their private segments must still be empty
AGPR_SPILL_OK = ["sim3opt_kernel", "mlpnp_quad_kernel"]


def test_hot_path_kernels_have_no_scratch():
    ks = _kernels()
    for frag in SCRATCH_FREE:
        hits = [n for n in ks if frag in n]
        assert hits, f"kernel {frag} not found in librsc.so"
        for n in hits:
            k = ks[n]
            assert k[".private_segment_fixed_size"] == 0, (n, k[".private_segment_fixed_size"])
            if not any(a in n for a in AGPR_SPILL_OK):
                assert k.get(".vgpr_spill_count", 0) == 0, (n, k[".vgpr_spill_count"])
