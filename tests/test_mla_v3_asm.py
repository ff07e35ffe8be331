"""Static check of the MLA v3 kernel's register discipline (csrc/ops/attn_mla.hip,
gen_mla_v3.py): the output accumulators are the literal AGPRs a[0:255], touched
only by generated inline asm, so the compiled variants must have no
hipcc-emitted v_accvgpr_* instruction, no scratch spills (bf16 and fp8 caches), and a generated
include that matches its generator."""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OPS = os.path.join(ROOT, "llmd_amd", "csrc", "ops")
HIPCC = "/opt/rocm/bin/hipcc"


def test_generated_include_is_current(tmp_path):
    gen = os.path.join(OPS, "gen_mla_v3.py")
    inc = os.path.join(OPS, "mla_v3_agpr.inc")
    before = open(inc).read()
    env = dict(os.environ)
    out = tmp_path / "copy"
    out.mkdir()
    shutil.copy(gen, out / "gen_mla_v3.py")
    subprocess.run([sys.executable, str(out / "gen_mla_v3.py")], check=True, capture_output=True, env=env)
    assert (out / "mla_v3_agpr.inc").read_text() == before


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_v3_accumulators_only_in_asm(tmp_path):
    s_path = tmp_path / "attn_mla.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17",
                    f"-I{os.path.join(ROOT, 'llmd_amd', 'csrc', 'include')}", "--cuda-device-only", "-S",
                    os.path.join(OPS, "attn_mla.hip"), "-o", str(s_path)], check=True, capture_output=True)
    s = s_path.read_text()
    names = re.findall(r"^(_ZN\S*mla_v3_kernelILb[01]ELb[01]ELb[01]E\S*):", s, re.M)  # BIG x fp8 x bf16-partials
    assert len(names) == 8
    v4 = re.findall(r"^(_ZN\S*mla_v4_kernelILb[01]ELb[01]E\S*):", s, re.M)  # the 32-key ring form
    assert len(v4) == 4
    names += v4
    for name in names:
        i = s.index(name + ":")
        j = s.index(".Lfunc_end", i)
        in_asm, stray, scratch = False, [], 0
        for line in s[i:j].split("\n"):
            if ";;#ASMSTART" in line:
                in_asm = True
            elif ";;#ASMEND" in line:
                in_asm = False
            elif not in_asm:
                op = line.strip().split(" ")[0]
                if "accvgpr" in op:
                    stray.append(line.strip())
                if op.startswith("scratch_"):
                    scratch += 1
        assert not stray, (name, stray[:5])
        assert scratch == 0, (name, scratch)


def test_prefill_v3_include_is_current(tmp_path):
    gen = os.path.join(OPS, "gen_prefill_v3.py")
    inc = os.path.join(OPS, "prefill_v3_agpr.inc")
    out = tmp_path / "copy"
    out.mkdir()
    shutil.copy(gen, out / "gen_prefill_v3.py")
    subprocess.run([sys.executable, str(out / "gen_prefill_v3.py")], check=True, capture_output=True)
    assert (out / "prefill_v3_agpr.inc").read_text() == open(inc).read()


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_prefill_v3_accumulators_only_in_asm(tmp_path):
    """attn_prefill.hip prefill_v3_kernel: O in a[0:127] (gen_prefill_v3.py), same audit."""
    s_path = tmp_path / "attn_prefill.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17",
                    f"-I{os.path.join(ROOT, 'llmd_amd', 'csrc', 'include')}", "--cuda-device-only", "-S",
                    os.path.join(OPS, "attn_prefill.hip"), "-o", str(s_path)], check=True, capture_output=True)
    s = s_path.read_text()
    names = re.findall(r"^(_ZN\S*prefill_v3_kernel\S*):", s, re.M)
    assert len(names) == 1
    i = s.index(names[0] + ":")
    j = s.index(".Lfunc_end", i)
    in_asm, stray, scratch = False, [], 0
    for line in s[i:j].split("\n"):
        if ";;#ASMSTART" in line:
            in_asm = True
        elif ";;#ASMEND" in line:
            in_asm = False
        elif not in_asm:
            op = line.strip().split(" ")[0]
            if "accvgpr" in op:
                stray.append(line.strip())
            if op.startswith("scratch_"):
                scratch += 1
    assert not stray, stray[:5]
    assert scratch == 0
