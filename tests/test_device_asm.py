"""Static checks of the gfx950 device code (CPU: hipcc cross-compiles)."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc not installed")
def test_no_valu_sgpr_to_vmem_hazard_in_inline_asm():
    """Every VMEM instruction that reads an SGPR written by a VALU instruction
    (a v_readlane reload of a spilled SGPR) sits at least 5 wait states after
    it.  hipcc resolves this hazard for its own code but not inside inline asm
    (the LDS-DMA control loads, the exchange step's record poll), which must
    carry its own s_nop; a record poll without one faulted on the GPU."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "asm_hazards.py")],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
