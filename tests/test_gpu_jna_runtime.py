"""GPU: the library in the JNA deployment configuration (no torch, /opt/rocm's ROCm).

Every other GPU test shares a process with torch, whose wheel bundles its own
libamdhip64 / librocfft / librccl (``_lib.load`` imports torch first so both use
one runtime).  A Java consumer has no torch: it binds the /opt/rocm stack the
library was linked against.  ``tests/jna_child.py`` is that process (numpy +
ctypes only); this test starts it fresh and requires every golden check to
match and /proc/self/maps to show /opt/rocm's runtime.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_jna_configuration_system_rocm_matches_golden(gpu):
    env = dict(os.environ, SPIMDECON_HIP_RUNTIME="system")
    r = subprocess.run([sys.executable, os.path.join(HERE, "jna_child.py")], capture_output=True, text=True,
                       timeout=300, env=env, cwd=os.path.dirname(HERE))
    print(r.stdout[-4000:])
    assert r.returncode == 0, (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert not res["failures"], res
    rocm = os.path.realpath("/opt/rocm")
    assert all(p.startswith(rocm + "/") for p in res["maps"]["libamdhip64.so"]), res["maps"]
    assert len([k for k in res["checks"] if k.startswith("rl_")]) >= 4, res["checks"]
