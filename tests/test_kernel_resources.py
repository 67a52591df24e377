"""Code-object checks of the shipped library (CPU only): the gfx950 kernels on the hot paths use no
scratch memory and spill no VGPRs.

A per-lane select written as `cond ? a[i + 1] : a[i]` over a register array can compile to a dynamic
index into scratch (round 4: the Hamming decode emission took 64 B of scratch per lane and ran 3x
slower); this catches that class of regression from the kernel descriptors alone, without a GPU.
The metadata comes from the library's offload bundles (llvm-objdump --offloading, then
llvm-readelf --notes on each gfx950 code object), extracted into a temporary directory."""
import os
import re
import shutil
import subprocess

import pytest
import yaml

LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "paritypartyfs_amd", "_lib",
                   "libppfs_ecc.so")

# hot-path kernels (name fragments of the mangled names): no scratch, no VGPR spills
HOT = ("rs_wg_encode_tk_kernel", "rs_wg_decode_tk_kernel", "rs_bs_encode_kernel", "ham_fast_encode_kernel",
       "ham_fast_decode_kernel", "crc_fast_encode_kernel", "crc_fast_check_kernel", "parity_fast")
# the cfg5 decode calls the general (2+ error) correction out of line: that call's frame is its only
# scratch (a fixed few dozen bytes, touched only by blocks with 2+ errors)
CALL_FRAME = {"rs_bs_decode_kernel": 128}


def kernel_descriptors(tmp_path):
    if not (os.path.exists(os.path.join(LLVM, "llvm-objdump")) and os.path.exists(os.path.join(LLVM, "llvm-readelf"))):
        pytest.skip("ROCm LLVM tools not found")
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    lib = tmp_path / "l.so"
    shutil.copy(LIB, lib)
    subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", str(lib)], cwd=tmp_path, check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    objs = sorted(p for p in os.listdir(tmp_path) if p.endswith("gfx950"))
    assert objs, "no gfx950 code object in the library"
    out = {}
    for o in objs:
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", o], cwd=tmp_path, check=True,
                               capture_output=True, text=True).stdout
        # the AMDGPU metadata is one YAML document ("---" ... "..."); read amdhsa.kernels[*] as YAML
        # so a kernel's fields are never confused with its arguments' (.args[*].name)
        m = re.search(r"^\s*---\s*$(.*?)^\s*\.\.\.\s*$", notes, re.S | re.M)
        assert m, f"no AMDGPU metadata in {o}"
        for kd in yaml.safe_load(m.group(1))["amdhsa.kernels"]:
            out[kd[".name"]] = {f: int(kd.get("." + f, 0)) for f in
                                ("private_segment_fixed_size", "vgpr_spill_count", "sgpr_spill_count", "vgpr_count")}
    return out


def test_hot_kernels_use_no_scratch(tmp_path):
    k = kernel_descriptors(tmp_path)
    hot = {n: d for n, d in k.items() if any(h in n for h in HOT)}
    assert len(hot) >= 10, sorted(k)
    bad = {n: d for n, d in hot.items() if d.get("private_segment_fixed_size", 0) or d.get("vgpr_spill_count", 0)}
    assert not bad, bad
    for frag, limit in CALL_FRAME.items():
        for n, d in k.items():
            if frag in n:
                assert d.get("private_segment_fixed_size", 0) <= limit and d.get("vgpr_spill_count", 0) == 0, (n, d)


# ------------------------------------------------------------------------------------------------
# Inline-asm hazard guard (round 4's r4b failure): a multi-instruction asm block that issues several
# memory reads from input address registers must mark its outputs early-clobber ("=&v").  Without
# it the register allocator may give a result the register of an address that a LATER read of the
# same block still needs -- the first read's data then overwrites the address before the next read
# issues (the t = 3 encode mismatched the oracle at 147,493 blocks on fc6e8df).
# ------------------------------------------------------------------------------------------------
CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "paritypartyfs_amd", "csrc")
READ_INSN = re.compile(r"\b(ds_read\w*|ds_load\w*|global_load\w*|buffer_load\w*|flat_load\w*|scratch_load\w*)")


def _asm_blocks(src):
    """(start line, template text, output constraints) of every asm statement in a source text."""
    out = []
    for m in re.finditer(r"\basm\s+(?:volatile\s*)?\(", src):
        i, depth, in_str, parts, cur = m.end(), 1, False, [], []
        while i < len(src) and depth:
            ch = src[i]
            if in_str:
                cur.append(ch)
                if ch == "\\":
                    cur.append(src[i + 1])
                    i += 1
                elif ch == '"':
                    in_str = False
            elif ch == '"':
                in_str = True
                cur.append(ch)
            elif ch == "(":
                depth += 1
                cur.append(ch)
            elif ch == ")":
                depth -= 1
                if depth:
                    cur.append(ch)
            elif ch == ":" and depth == 1:
                parts.append("".join(cur))
                cur = []
            else:
                cur.append(ch)
            i += 1
        parts.append("".join(cur))
        template = "".join(re.findall(r'"((?:[^"\\]|\\.)*)"', parts[0]))
        template = template.replace("\\n", "\n").replace("\\t", "\t")  # instruction separators
        outputs = re.findall(r'"(=[^"]*|\+[^"]*)"', parts[1]) if len(parts) > 1 else []
        out.append((src.count("\n", 0, m.start()) + 1, template, outputs))
    return out


def asm_clobber_violations(src):
    bad = []
    for line, template, outputs in _asm_blocks(src):
        if len(READ_INSN.findall(template)) < 2:
            continue
        late = [o for o in outputs if o.startswith("=") and not o.startswith("=&")]
        if late:
            bad.append((line, late))
    return bad


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".hip", ".cpp")))


def test_multi_read_asm_blocks_use_early_clobber_outputs():
    seen = 0
    for path in _sources():
        src = open(path).read()
        seen += sum(len(READ_INSN.findall(t)) >= 2 for _, t, _ in _asm_blocks(src))
        assert not asm_clobber_violations(src), (os.path.basename(path), asm_clobber_violations(src))
    assert seen >= 2, "the multi-read asm blocks (rs_wg_tk.hpp win5x1 / win5x3) were not found"


def test_clobber_guard_catches_the_r4b_regression():
    """Positive control: win5x3 with its outputs reverted to plain "=v" is flagged."""
    src = open(os.path.join(CSRC, "rs_wg_tk.hpp")).read()
    assert not asm_clobber_violations(src)
    start = src.index("void win5x3(")
    broken = src[:start] + src[start:].replace('"=&v"', '"=v"', 9)
    assert asm_clobber_violations(broken)
