"""Runtime scheduling variants, each in a child process whose legacy RT_* environment switches
tests/helpers.make_renderer maps onto the library's rt_set_tuning / rt_set_graphs (the library
itself reads no environment): host-driven rounds (RT_WF_HOST=1: queue sizes read back every round instead of
the device-side round control), eager enqueue without frame graphs (RT_GRAPH=0), and the finish
kernel's scheduling knobs at other values (odd chunk sizes, an absolute shading threshold after the
queue runs out, the long-first order's chunks split over few blocks, the finish drain's team
sizes: 2, 4 and 8 lanes, and off, which these small frames (< 256K paths) use by default), against the committed golden fixtures (bit-identical radiance, depth and ray counts).  The bulk pipelines run
wf_shade every bounce (the small fixture frames would otherwise go straight to the finish kernel)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = "c3g_small_b8,c1_ema_f3,lights_mix4_b3,c2_small_b4"
PIPES = "wavefront,wavefront-bulk,wavefront-mixed"


@pytest.mark.parametrize("env", [{"RT_WF_HOST": "1"}, {"RT_GRAPH": "0"},
                                 {"RT_FCHUNK": "7", "RT_SHADE_MIN_X": "24", "RT_FINISH_FRAC": "1"},
                                 {"RT_FCHUNK": "1", "RT_SHADE_MIN_X": "-100", "RT_SHADE_MIN": "1"},
                                 {"RT_TEAM": "2"}, {"RT_TEAM": "4"}, {"RT_TEAM": "8", "RT_FCHUNK": "3"}, {"RT_TEAM": "0"},
                                 ],
                         ids=["hostrounds", "nograph", "finish_chunk7", "finish_chunk1", "team2", "team4", "team8", "noteam"])
def test_env_variant_matches_golden(env):
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "env_variant_child.py"), CASES, PIPES], env=e,
                       capture_output=True, text=True, timeout=150)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert r.stdout.count(" ok ") == len(CASES.split(",")) * len(PIPES.split(","))
