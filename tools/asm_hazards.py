"""Scan the HIP library's gfx950 device assembly for one hazard hipcc does not
resolve inside inline asm: a VALU instruction that writes an SGPR (typically
the v_readlane reload of a spilled SGPR) followed, within 5 wait states, by a
VMEM instruction that reads that SGPR (the `saddr` base of the LDS-DMA and
record loads).  CDNA needs 5 wait states there; with fewer the load may use
the SGPR's previous value — a wrong address (measured: an illegal-address
fault).
    python tools/asm_hazards.py [file.s]     (default: compile mpc_rollout.hip)
Exit status 1 and one line per hazard if any is found."""
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WAITS = 5


def device_asm():
    out = os.path.join(tempfile.mkdtemp(), "mpc_rollout.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                    "-ffp-contract=off", "-I", os.path.join(REPO, "include"),
                    "--cuda-device-only", "-S", "-o", out,
                    os.path.join(REPO, "diplomjourney_amd", "csrc", "mpc_rollout.hip")],
                   check=True, capture_output=True, cwd=tempfile.gettempdir())
    return out


def sgprs(tok):
    m = re.match(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"s(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def is_insn(line):
    return bool(line) and not line.startswith((";", ".")) and not line.endswith(":")


def scan(lines):
    hits = []
    func = "?"
    for n, raw in enumerate(lines):
        m = re.match(r"^(_Z[^:]+):", raw)
        if m:
            func = m.group(1)
        t = raw.strip()
        if not t.startswith(("global_", "buffer_", "scratch_")) or " " not in t:
            continue
        used = set()
        for op in t.split(None, 1)[1].split(","):
            op = op.strip()
            if op:
                used |= sgprs(op.split()[0])
        if not used:
            continue
        k, waits = n - 1, 0
        while k >= 0 and waits < WAITS:
            u = lines[k].strip()
            k -= 1
            if not is_insn(u):
                continue
            parts = u.split(None, 1)
            if parts[0] == "s_nop":
                waits += int(parts[1], 0) + 1 if len(parts) > 1 else 1
                continue
            if parts[0].startswith("v_") and len(parts) > 1 and sgprs(parts[1].split(",")[0].strip()) & used:
                hits.append(f"{func}: `{t}` {waits} wait state(s) after `{u}`")
            waits += 1
    return hits


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else device_asm()
    hits = scan(open(path).read().splitlines())
    for h in hits:
        print(h)
    print(f"{len(hits)} VALU-SGPR -> VMEM hazard(s)")
    return 1 if hits else 0


if __name__ == "__main__":
    sys.exit(main())
