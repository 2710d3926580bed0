"""The shipped gfx950 code object, disassembled on the CPU.

Round 3 traced rare label-map mismatches of concurrent plan copies to packed-f32 VALU
results (``v_pk_fma_f32`` / ``v_pk_mul_f32`` / ``v_pk_add_f32``) coming back wrong under
co-residence with other kernels' waves (profiles/r3_packed_f32_race.txt) and builds the
HIP extension without packed-f32 ops (``ops/build.py``: ``-target-feature
-packed-fp32-ops``). This test unbundles every gfx950 code object inside the built
extension's ``.hip_fatbin`` section and asserts that none of them contains a packed-f32
instruction, so a flag change or a kernel built another way cannot silently bring the
instructions back. It also checks that the kernels are really MFMA code."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _so():
    import sysconfig
    return os.path.join(ROOT, "semantic_segmentation_server_amd", "ops",
                        "_hip" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))


def _tools_ok():
    return all(os.path.exists(os.path.join(LLVM, t)) for t in ("clang-offload-bundler", "llvm-objdump")) \
        and shutil.which("objcopy") is not None


def code_objects(so_path, workdir):
    """The gfx950 code objects of every offload bundle in the .hip_fatbin section."""
    fat = os.path.join(workdir, "fat.bin")
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", so_path, os.path.join(workdir, "x.so")],
                   check=True, capture_output=True)
    data = open(fat, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    assert starts, "no offload bundle in .hip_fatbin"
    out = []
    for i, s in enumerate(starts):
        e = starts[i + 1] if i + 1 < len(starts) else len(data)
        b = os.path.join(workdir, f"b{i}.bin")
        with open(b, "wb") as f:
            f.write(data[s:e])
        co = os.path.join(workdir, f"co{i}.o")
        r = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                            f"--input={b}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"],
                           capture_output=True, text=True)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            out.append(co)
    return out


@pytest.mark.skipif(not _tools_ok(), reason="ROCm LLVM tools not present")
def test_no_packed_f32_in_shipped_code_object(tmp_path):
    so = _so()
    if not os.path.exists(so):
        pytest.skip("HIP extension not built (run __graft_entry__.build())")
    cos = code_objects(so, str(tmp_path))
    assert cos, "no gfx950 code object found"
    n_pk, n_mfma = 0, 0
    offenders = {}
    for co in cos:
        dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co],
                             capture_output=True, text=True, check=True).stdout
        fn = None
        for line in dis.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
            if m:
                fn = m.group(1)
                continue
            if re.search(r"\bv_pk_(fma|mul|add)_f32\b", line):
                n_pk += 1
                offenders[fn] = offenders.get(fn, 0) + 1
            elif "v_mfma_" in line:
                n_mfma += 1
    assert n_pk == 0, f"packed-f32 VALU in the shipped code object: {offenders}"
    assert n_mfma > 1000, n_mfma  # the model / ASPP / int8 kernels are MFMA code
