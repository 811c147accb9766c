"""No kernel of libvaesne_hip contains a packed-FP32 VALU op that reads the high half of a
VGPR source into its low lane (v_pk_{fma,mul,add}_f32 with an op_sel bit set on a VGPR
operand).  Measured unaffected, and so allowed: an SGPR-pair source (hipcc's scalar-broadcast
multiplies), v_pk_mov_b32 with op_sel (hipcc's register shuffles), op_sel_hi.

On gfx950 such an op returns wrong values while another wave on the same CU runs
v_mfma_f32_16x16x32_{f16,bf16} (tools/probe/mfma_interference.py: 5-17 % of the lanes of a
plain op_sel:[0,1,0] FMA chain wrong beside an f16 MFMA loop, none without it, none with
op_sel_hi only; DESIGN.md "A packed-FP32 erratum").  The split-f16 attention kernels run
that MFMA on one stream while the packed-VALU kernels (the decoders' first-block
attention) and the elementwise kernels run on the others, so the library must not contain
the form at all.  CPU-only: the device code objects are unbundled from the build's objects
and disassembled."""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
PK = re.compile(r"^\s*(v_pk_(?:fma|mul|add)_f32)\s+([^/]*?)\s*(?:op_sel:\[([01,]+)\])")


def _violations(line):
    """the VGPR source operands of a packed op whose op_sel bit is set"""
    m = PK.search(line)
    if not m:
        return []
    ops = [o.strip() for o in m.group(2).split(",")]
    srcs = ops[1:]                              # ops[0] is the destination
    bits = [b == "1" for b in m.group(3).split(",")]
    return [src for src, b in zip(srcs, bits) if b and src.startswith("v")]


def _objects():
    sys.path.insert(0, os.path.join(ROOT, "vaesne-dev_amd"))
    import build_lib
    build_lib.build(verbose=False)
    return [build_lib._compile(src) for src in build_lib.sources()]   # up to date: no rebuild


@pytest.mark.skipif(not os.path.exists(os.path.join(LLVM, "llvm-objdump")), reason="no ROCm llvm tools")
def test_no_low_lane_high_half_packed_fp32(tmp_path):
    objs = _objects()
    assert objs, "no objects built"
    bad = []
    for o in objs:
        fat, co = tmp_path / (os.path.basename(o) + ".fat"), tmp_path / (os.path.basename(o) + ".co")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", o,
                        str(tmp_path / "stripped.o")], check=True, capture_output=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}", "--unbundle"],
                       check=True, capture_output=True)
        dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", str(co)],
                             check=True, capture_output=True, text=True).stdout
        assert "v_" in dis, f"no device code disassembled from {o}"
        for line in dis.splitlines():
            if _violations(line):
                bad.append((os.path.basename(o), line.strip()))
    assert not bad, f"{len(bad)} packed-FP32 ops read a VGPR's high half into the low lane, e.g. {bad[:3]}"


def test_violation_parser():
    assert _violations("v_pk_fma_f32 v[2:3], v[4:5], v[6:7], v[2:3] op_sel:[0,1,0] op_sel_hi:[1,1,1]") == ["v[6:7]"]
    assert _violations("v_pk_mul_f32 v[76:77], s[8:9], v[54:55] op_sel:[1,0]") == []
    assert _violations("v_pk_fma_f32 v[2:3], v[4:5], v[6:7], v[2:3] op_sel_hi:[1,0,1]") == []
    assert _violations("v_pk_add_f32 v[8:9], v[4:5], v[6:7] op_sel:[1,0] op_sel_hi:[0,1]") == ["v[4:5]"]


def test_step_torch_kernels_free_of_the_form():
    """The aten kernels the captured training step runs (the latest committed kernel trace,
    profiles/LATEST/kernel_stats.csv) are none of the torch kernels whose gfx950 code holds
    the form: profiles/r06/isa_scan_torch.json lists them, from tools/isa_scan_torch.py's
    disassembly of every offload bundle of libtorch_hip.so (829 of 23854 symbols, e.g.
    complex-float elementwise and bf16 norm reductions).  Matching is by exact kernel name
    (whitespace-normalised).  A different torch build invalidates the scan: skipped then."""
    import csv
    import json
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_scan_torch
    scan = json.load(open(os.path.join(ROOT, "profiles", "r06", "isa_scan_torch.json")))
    try:
        lib = isa_scan_torch.torch_hip_lib()
        if os.path.getsize(lib) != scan["lib_size"]:
            pytest.skip("torch differs from the scanned build: rerun tools/isa_scan_torch.py")
    except OSError:
        pytest.skip("no libtorch_hip")
    latest = open(os.path.join(ROOT, "profiles", "LATEST")).read().strip()
    names = [r["Name"] for r in csv.DictReader(open(os.path.join(ROOT, "profiles", latest, "kernel_stats.csv")))]
    aten, hit = isa_scan_torch.match_trace(scan["kernels"], names)
    assert aten, "the trace should hold some aten kernels (copies, fills)"
    assert not hit, f"aten kernels of the step carry the erratum form: {list(hit)[:3]}"
    # the matcher itself: a scanned name matches its trace spelling ("> >" vs ">>")
    k = next(iter(scan["kernels"]))
    assert isa_scan_torch.match_trace(scan["kernels"], [k.replace(">>", "> >")])[1]
