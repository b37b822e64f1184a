"""Every traversal instance on adversarial closest-hit geometry (VERDICT r4 'what's weak' 1): the
triangle soup (overlapping triangles whose ids say nothing about their depth: round 3's stale
second-triangle bound kept a farther hit there) and the exact-tie scene (bit-identical duplicate
triangles under different materials, a rotated copy, a quad grid with shared edges: only the
min-id tie-break of DESIGN.md §4 picks the material), against the CPU oracle (Raytracing.metal:
301-322 closest hit, :716-743 any hit).

Instances: wf_trace (the bulk pipeline: every bounce through extend / connect launches), the plain
finish kernel (wf_finish_step: the whole small frame goes to the finish), its team drain at 2, 4
and 8 lanes per query (RT_TEAM; RT_FCHUNK=1 makes every wave's paths few, so the drain engages at
once).  The 512x512 frames (262,144 base paths) sit
inside the team drain's default range (kTeamAutoMin .. kTeamAutoPaths), so its default instance
runs there without any switch."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
SMALL = "soup:64:48:2:3,ties:64:48:2:3"
PIPES = "wavefront,wavefront-bulk,wavefront-mixed"


def _run(env, specs, pipes):
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "traversal_variant_child.py"), specs, pipes], env=e,
                       capture_output=True, text=True, timeout=240)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert r.stdout.count(" ok ") == len(specs.split(",")) * len(pipes.split(","))


@pytest.mark.parametrize("env", [{}, {"RT_TEAM": "0"}, {"RT_TEAM": "2", "RT_FCHUNK": "1"}, {"RT_TEAM": "4", "RT_FCHUNK": "1"},
                                 {"RT_TEAM": "8", "RT_FCHUNK": "1"}, {"RT_TEAM": "4", "RT_FCHUNK": "5", "RT_SHADE_MIN_X": "1"},
                                 ],
                         ids=["default", "noteam", "team2", "team4", "team8", "team4_chunk5"])
def test_traversal_instances_small(env):
    _run(env, SMALL, PIPES)


@pytest.mark.parametrize("env", [{}, {"RT_TEAM": "2"}, {"RT_TEAM": "8"}, {"RT_TEAM": "0"}],
                         ids=["default_team4", "team2", "team8", "noteam"])
def test_traversal_instances_team_range(env):
    """512 x 512 x 1 spp, 3 bounces: 262,144 base paths, the default team drain's range."""
    _run(env, "soup:512:512:1:3,ties:512:512:1:3", "wavefront")
