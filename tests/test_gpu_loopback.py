"""ptx_comm.cpp's RCCL exchange with N > 1 ranks, on one GPU.

Real RCCL refuses two ranks on one device, so the handle-owned communicator path
(render_band_nccl: grouped ncclSend / ncclRecv of the static halo and the motion halo,
pipelined band frames, check_neighbours, comm_health, the failure and teardown paths) never ran
with N > 1 before the driver's 8-GPU bench.  Here libptx.so dlopens the in-process loopback
communicator instead (PTX_RCCL_LIB = tests/loopback/libptx_loopback_rccl.so, whose send / recv
are stream-ordered device copies) and four band handles on one GPU run that exact code, each
from its own host thread as separate ranks would.  The script runs in a child process
(tests/loopback_bands.py): the RCCL library is chosen once per process.

Checked: along the 8-frame moving-camera path plus a 12-degree pitch turn (past the R-row motion
halo: the motion rule clips those reprojections in every handle) and three frames through
ptx_render_bands' communicator branch, the 4-band split equals one handle bit for bit (temporal
output, spatial output, radiance) after every frame; both count the same clipped pixels; a rank
that reset its history while the camera moves does not desynchronise the exchange; ReSTIR GI's
motion pass over three communicator bands equals one handle too; a rank whose peer never renders
gets an error status within the deadline and its communicator is aborted.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "tests", "loopback", "libptx_loopback_rccl.so")


@pytest.mark.gpu
def test_loopback_communicator_bands():
    assert os.path.exists(STUB), "build it: make -C tests/loopback (or __graft_entry__.build())"
    env = dict(os.environ, PTX_RCCL_LIB=STUB, LOOPBACK_TIMEOUT_MS="3000", PTX_AB="COMM_TIMEOUT_S=10")
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "loopback_bands.py")], env=env,
                       capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    sp = out["split"]
    for fr in sp["frames"]:
        assert fr["history"] == fr["temporal"] == fr["radiance"] == 0, fr
    assert len(sp["frames"]) == 13 and any(fr.get("render_bands") for fr in sp["frames"])
    assert sp["clips_one"] > 0 and sp["clips_bands"] == sp["clips_one"]
    assert sp["hist_used"] > 0.2
    assert all(c["world"] == 4 and c["halo_bytes_sent"] > 0 for c in sp["comm"])
    gi = out["gi_split"]
    for fr in gi["frames"]:
        assert fr["history"] == fr["temporal"] == fr["radiance"] == 0, fr
    assert gi["clips_one"] > 0 and gi["clips_bands"] == gi["clips_one"]
    assert gi["hist_used"] > 0.2
    rr = out["reset_one_rank"]
    assert all(not any(e) for e in rr["errors"]), rr
    assert rr["finite"]
    dp = out["dead_peer"]
    assert dp["error"] and dp["seconds"] < 30, dp
    assert dp["aborts"] == 1 and dp["destroys_healthy"] == 1, dp
    st = out["stub"]
    assert st["pairs"] > 100 and st["bytes"] > 0
