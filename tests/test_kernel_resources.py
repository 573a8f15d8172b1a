"""Register and LDS budgets of the product's gfx950 kernels, read from the built
library's code objects (no GPU): the kernels that carry the measured lines run
without scratch spills, and the 12-site light-cone end fits four workgroups per
CU.  Round 6 found 30 pass kernels spilling 12-100 B per thread (an 8-B store
offset or slot base kept alive through the pass at the VGPR cap; the 12-site
end's spill alone wrote 273 MB of scratch per launch, profiles/r6f); this
keeps those fixes from regressing silently."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "noise-resilience-in-discrete-time-crystal-realizations-on-quantum-computers_amd",
                   "lib", "libdtc_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# demangled name -> what it carries (BASELINE configs / bench.py lines)
MEASURED = {
    "dtc::dtc_kdk_pass3<7, 0, 0, 0>": "C2 12-site K-D-K",
    "dtc::dtc_kdk_pass<6, 0, 0, 0>": "C2 8-site K-D-K",
    "dtc::dtc_kdk_dual<7, 0, 1, 0>": "C2 dual pass, 12-site",
    "dtc::dtc_kdk_dual<6, 0, 1, 0>": "C2 dual pass, 8-site",
    "dtc::dtc_lcw3_final<0>": "C2 12-site light-cone end",
    "dtc::dtc_lcw2_final<0>": "C2 10-site light-cone end",
    "dtc::dtc_kdk_pass3<7, 3, 0, 0>": "C3 12-site device-noise K-D-K",
    "dtc::dtc_kdk_pass<6, 3, 0, 0>": "C3 8-site device-noise K-D-K",
    "dtc::dtc_kdk_dual<7, 3, 1, 0>": "C3 dual pass, 12-site",
    "dtc::dtc_kdk_dual<6, 3, 1, 0>": "C3 dual pass, 8-site",
    "dtc::dtc_kdk_pass3<6, 0, 2, 0>": "C4 per-site K-D-K",
    "dtc::dtc_kick_pass<7, 0, 0, 0>": "C4 / C5 kick-only pass",
    "dtc::dtc_kick_swap_pass<6, 0>": "C5 fused kick + exchange",
    "dtc::dtc_kdk_pass3<7, 0, 3, 0>": "energy 12-site pass",
    "dtc::dtc_kdk_pass3<6, 0, 3, 0>": "energy 8-site pass",
}


def _kernels():
    tools = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf")]
    if not os.path.exists(LIB) or not all(os.path.exists(t) for t in tools) or not shutil.which("c++filt"):
        pytest.skip("built library or ROCm LLVM tools missing")
    objcopy, bundler, readelf = tools
    out = {}
    tmp = os.path.join(ROOT, "build", "kres")
    os.makedirs(tmp, exist_ok=True)
    fat = os.path.join(tmp, "fatbin")
    subprocess.run([objcopy, "--dump-section", ".hip_fatbin=" + fat, LIB, os.path.join(tmp, "lib.so")],
                   check=True, capture_output=True)
    data = open(fat, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    for i, s in enumerate(starts):
        part = os.path.join(tmp, f"bundle{i}")
        with open(part, "wb") as f:
            f.write(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
        co = part + ".co"
        r = subprocess.run([bundler, "--unbundle", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                            "--input=" + part, "--output=" + co], capture_output=True)
        if r.returncode != 0 or not os.path.exists(co) or os.path.getsize(co) == 0:
            continue
        notes = subprocess.run([readelf, "--notes", co], capture_output=True, text=True).stdout
        cur = {}
        for line in notes.splitlines():
            m = re.match(r"\s+\.(name|private_segment_fixed_size|group_segment_fixed_size|vgpr_count):\s+(\S+)",
                         line)
            if not m:
                continue
            key, val = m.groups()
            if key == "name":
                cur = out.setdefault(val, {})
            else:
                cur[key] = int(val)
    if not out:
        pytest.skip("no gfx950 code objects found in the library")
    names = list(out)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    return {d.replace("void ", "").split("(")[0]: out[n] for n, d in zip(names, dem)}


def test_measured_kernels_do_not_spill():
    k = _kernels()
    missing = [n for n in MEASURED if n not in k]
    assert not missing, missing
    spills = {n: k[n]["private_segment_fixed_size"] for n in MEASURED if k[n].get("private_segment_fixed_size")}
    assert not spills, {n: (MEASURED[n], b) for n, b in spills.items()}


def test_lcw3_fits_four_workgroups_per_cu():
    k = _kernels()["dtc::dtc_lcw3_final<0>"]
    # 160 KiB of LDS per CU / 4 and 512 VGPRs per SIMD lane / 4 waves (the
    # fourth workgroup is worth more than any instruction cut that costs LDS, r6y)
    assert k["group_segment_fixed_size"] <= 160 * 1024 // 4
    assert k["vgpr_count"] <= 128
