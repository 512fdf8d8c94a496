"""Build guard (randblas_amd/csrc/Makefile): fail when a streamed GEMM kernel whose memory ring is
loaded by inline asm spills registers.

skge_stream_kernel's one-triangle and transposed operand forms (template TRI 1-5) issue their ring
loads as inline asm with "=v" outputs and wait for them later (s_waitcnt vmcnt(N) + vm_fence). The
compiler takes such a register as written when the asm issues, so a spill or copy of a ring register
between the load and its wait would move the value before the data has landed -- wrong results, and
no test of a different shape would see it. (Round 5's RBH_TRI_WIDE build spilled 24-64 B a lane in
exactly these kernels and failed the bitwise suite.) The compiler's resource remarks
(-Rpass-analysis=kernel-resource-usage) list ScratchSize and VGPR spills per kernel; this script reads
them, echoes the compiler's other diagnostics, and exits 1 if any such kernel spills.

usage: check_spills.py REMARKS_FILE
"""
import re
import sys


def kernels(lines):
    """{mangled kernel name: {remark key: value}} from the resource-usage remarks."""
    out, cur = {}, None
    for line in lines:
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z][A-Za-z /\[\]]*?):\s+(\S+) \[-Rpass-analysis", line)
        if m and cur:
            out[cur][m.group(1).strip()] = m.group(2)
    return out


def stream_tri(name):
    """TRI (the last template argument) of a skge_stream_kernel instantiation, or None."""
    m = re.search(r"skge_stream_kernelI[df]((?:L[ib]\d+E)+)E", name)
    if not m:
        return None
    return int(re.findall(r"L[ib](\d+)E", m.group(1))[-1])


def main(path):
    with open(path) as f:
        lines = f.readlines()
    for line in lines:   # the compiler's warnings and errors, as a normal build shows them
        # (a remark's source excerpt follows it: "  292 | code" and "      | ^")
        if ("-Rpass-analysis=kernel-resource-usage" not in line and line.strip()
                and not re.match(r"^\s*(\d+\s*)?\|", line)):
            sys.stderr.write(line)
    bad = []
    for name, r in kernels(lines).items():
        tri = stream_tri(name)
        if tri is None or tri == 0:
            continue
        scratch = int(r.get("ScratchSize [bytes/lane]", "0"))
        spill = int(r.get("VGPRs Spill", "0"))   # (SGPR spills go to VGPR lanes, not the ring)
        if scratch or spill:
            bad.append((name, scratch, spill))
    for name, scratch, spill in bad:
        sys.stderr.write(f"check_spills: {name}: scratch {scratch} B/lane, {spill} spilled registers -- its "
                         f"asm-loaded ring is unsafe\n")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
