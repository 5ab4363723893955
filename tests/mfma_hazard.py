"""MFMA result-read hazard check over the gfx950 code objects of libpghip.so (test aid, VERDICT r5 "What's weak" 8).

Round 5 found hipcc sinking a v_mfma chain into a guarded epilogue block and reading the first accumulator register a
few instructions after the last MFMA on the branch-skipping path, inside the MFMA's write latency
(profiles/r05_mfma_sink_hazard.txt).  This scans every kernel of the library: for each v_mfma* it walks every
instruction path that follows it (fall-through and branch targets) for the MFMA's required wait states and reports any
instruction that reads one of the MFMA's destination registers before they have elapsed.

Wait-state model (the one the compiler's hazard recognizer uses): each instruction is one wait state, `s_nop N` is N+1.
Required between an XDL MFMA and a non-MFMA read of its result (VALU, memory, LDS, v_accvgpr_read) or its use as
an MFMA's A/B operand: passes + 3 (gfx940's passes + 2, one more on gfx950), passes = 4 for v_mfma_f32_16x16x32_bf16
and 8 for v_mfma_scale_f32_16x16x128_f8f6f4 (twice its cycles, MI355X_MICROARCH.md § Matrix cores).  An MFMA reading
the register as its accumulator (srcC) is the hardware's back-to-back accumulation path and is not counted.
"""
from __future__ import annotations

import os
import re
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
PASSES = {"v_mfma_f32_16x16x32_bf16": 4, "v_mfma_scale_f32_16x16x128_f8f6f4": 8,
          "v_mfma_f32_32x32x16_bf16": 8, "v_mfma_scale_f32_32x32x64_f8f6f4": 16}
DEFAULT_PASSES = 16          # an MFMA opcode not in the table: the longest

_REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")
_LINE = re.compile(r"^\s+([a-z_0-9]+)(?:\s+(.*?))?\s*//\s*([0-9A-Fa-f]+):")
_LABEL = re.compile(r"^([0-9a-fA-F]+) <([^>]+)>:")
_TARGET = re.compile(r"<([^>+]+)(?:\+0x([0-9a-fA-F]+))?>")


def code_objects(lib: str) -> list[bytes]:
    """The gfx950 code objects of every bundle in lib's .hip_fatbin (one per translation unit)."""
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", lib, os.path.join(d, "x")],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
        offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
        out = []
        for i in range(len(offs) - 1):
            b = os.path.join(d, f"b{i}.fat")
            co = os.path.join(d, f"b{i}.co")
            with open(b, "wb") as f:
                f.write(data[offs[i]:offs[i + 1]])
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={b}", f"--output={co}",
                                "--unbundle"], capture_output=True)
            if r.returncode == 0 and os.path.getsize(co) > 0:
                out.append(open(co, "rb").read())
        return out


def disassemble(co: bytes) -> str:
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", f.name], check=True,
                              capture_output=True, text=True).stdout


def _regs(text: str) -> set:
    s = set()
    for m in _REG.finditer(text):
        kind = m.group(1)
        if m.group(4) is not None:
            s.add((kind, int(m.group(4))))
        else:
            for r in range(int(m.group(2)), int(m.group(3)) + 1):
                s.add((kind, r))
    return s


def _split_ops(ops: str) -> list[str]:
    out, depth, cur = [], 0, ""
    for ch in ops:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def _reads(op: str, ops: list[str]) -> set:
    """Registers an instruction reads (a conservative split of destination and sources)."""
    if op.startswith("v_mfma"):
        return _regs(" ".join(ops[1:3]))                      # srcA, srcB (srcC: accumulation, not counted)
    if op.startswith("s_"):
        return set()
    store = ("store" in op or "write" in op or "atomic" in op) and not op.startswith("v_")
    if store:
        return _regs(" ".join(ops))
    return _regs(" ".join(ops[1:]))                           # first operand is the destination


def parse(text: str):
    """-> (instructions [(addr, op, ops, kernel)], index by address, kernel start addresses)."""
    ins, kernels, cur = [], {}, None
    for line in text.splitlines():
        m = _LABEL.match(line)
        if m:
            cur = m.group(2)
            kernels[cur] = int(m.group(1), 16)
            continue
        m = _LINE.match(line)
        if m and cur is not None:
            ops = _split_ops(m.group(2) or "")
            ins.append((int(m.group(3), 16), m.group(1), ops, cur, line))
    index = {a: i for i, (a, *_r) in enumerate(ins)}
    return ins, index, kernels


def _branch_target(raw: str, kernels: dict):
    m = _TARGET.search(raw)
    if not m or m.group(1) not in kernels:
        return None
    return kernels[m.group(1)] + int(m.group(2) or "0", 16)


def find_hazards(text: str, limit: int = 50) -> tuple[list, int]:
    """Every (kernel, mfma address, reading instruction, wait states elapsed, required) where a path reads an MFMA
    result too early; and the number of MFMAs checked."""
    ins, index, kernels = parse(text)
    bad, n_mfma = [], 0
    for i, (addr, op, ops, kern, _raw) in enumerate(ins):
        if not op.startswith("v_mfma"):
            continue
        n_mfma += 1
        need = PASSES.get(op, DEFAULT_PASSES) + 3
        dst = _regs(ops[0]) if ops else set()
        # DFS over paths: (instruction index, wait states elapsed)
        stack, seen = [(i + 1, 0)], set()
        while stack:
            j, w = stack.pop()
            while j < len(ins) and w < need:
                if (j, w) in seen:
                    break
                seen.add((j, w))
                a2, op2, ops2, k2, raw2 = ins[j]
                if k2 != kern:
                    break
                if _reads(op2, ops2) & dst:
                    bad.append((kern, hex(addr), raw2.split("//")[0].strip(), w, need))
                    break
                if op2.startswith("v_mfma") and _regs(ops2[0] if ops2 else "") & dst:
                    break                                     # overwritten by a later MFMA: its own hazard window
                if op2 == "s_nop":
                    w += int(ops2[0], 0) + 1 if ops2 else 1
                else:
                    w += 1
                if op2 == "s_endpgm" or op2.startswith("s_setpc"):
                    break
                if op2.startswith("s_cbranch") or op2 == "s_branch":
                    t = _branch_target(raw2, kernels)
                    if t is not None and t in index:
                        stack.append((index[t], w))
                    if op2 == "s_branch":
                        break
                j += 1
        if len(bad) >= limit:
            break
    return bad, n_mfma
