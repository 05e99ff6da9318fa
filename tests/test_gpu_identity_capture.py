"""GPU: the identity-loss side stream inside a whole-step hipGraph.

BASELINE configs[2] (bs32, ResNet-50 identity-preserving loss, FeatureExtract.py /
ResNet.py) runs the frozen extractor's forward and input-gradient backward on a side HIP
stream (tpgan_train.IDENTITY_STREAM).  Round 5 saw the process crash when such a fork ran in
eager steps and the whole step was then captured and replayed under bench.py's graph
environment (packet capture off, 8 graph queues).  This runs exactly that sequence in a child
process with bench.py's environment -- eager steps with the fork, one unsegmented capture with
the fork inside it, replays -- and requires the replays to equal the eager steps bit for bit
(deterministic mode)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_identity_fork_whole_step_capture_bs32_resnet50(gpu):
    env = dict(os.environ, DEBUG_CLR_GRAPH_PACKET_CAPTURE="0", DEBUG_HIP_FORCE_GRAPH_QUEUES="8",
               PYTHONFAULTHANDLER="1")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tests", "_identity_capture_run.py"), "32"], cwd=REPO,
                       env=env, capture_output=True, text=True, timeout=580)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-5000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["graphs"] == 1 and out["fork_in_capture"], out
    assert out["G_equal"] and out["D_equal"], out
    assert out["losses"] == out["losses_eager"], out
