"""Seed inputs for tools/fuzz_host.cpp: the skinned test asset of tests/test_usd.py as .usda,
.usdc and .usdz (crate + PNG texture), and the test PNG.  Usage: python tools/fuzz_seeds.py DIR"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import usd_writers as W  # noqa: E402
from test_usd import TEX, robot_prims  # noqa: E402

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
prims, _ = robot_prims()
# + an internal reference, and a variant set whose selected variant spec references it again
crate = W.write_usdc(prims + [dict(path="/Copy", type="Xform", refs=[("", "/Robot/Prop")]),
                              dict(path="/Var", type="Xform", variant_sets={"v": ["a", "b"]}, variant_sel={"v": "b"}),
                              dict(path="/Var{v=a}"), dict(path="/Var{v=b}"),
                              dict(path="/Var{v=b}/Again", type="Xform", refs=[("", "/Robot/Prop")])])
files = {
    # + composition: an internal reference and a variant set whose selected body references it again
    "seed.usda": W.write_usda(prims) + b"""
def Xform "World" (
    variants = {
        string lod = "full"
    }
    prepend variantSets = "lod"
)
{
    def "Copy" (
        prepend references = </Robot/Prop>
    )
    {
    }
    variantSet "lod" = {
        "full" {
            def "Again" (
                references = </Robot>
            )
            {
            }
        }
        "proxy" {
        }
    }
}
""",
    # internal-reference fan-out over a layer holding one large array (every internal
    # arc's layer snapshot is charged against the composed-bytes budget)
    "seed_fanout.usda": b"#usda 1.0\n"
    + b'def Mesh "Src"\n{\n    int[] faceVertexCounts = [3]\n    int[] faceVertexIndices = [0, 1, 2]\n'
    + b"    point3f[] points = [" + b", ".join(b"(%d, %d, 1)" % (i, i % 7) for i in range(4096)) + b"]\n}\n"
    + b'def Xform "Tiny"\n{\n}\n'
    + b"".join(b'def Xform "R%d" (\n    references = </Tiny>\n)\n{\n}\n' % i for i in range(256)),
    "seed.usdc": crate,
    "seed.usdz": W.write_usdz("robot.usdc", crate, [("textures/tex.png", TEX)]),
    "seed.png": TEX,
    # a quad and a triangle with normals, texture coordinates, negative indices and a polygon
    "seed.obj": b"""# fuzz seed
o quad
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
v 0.5 1.5 0.2
vn 0 0 1
vt 0 0
vt 1 0
vt 1 1
vt 0 1
f 1/1/1 2/2/1 3/3/1 4/4/1
f -1 -2 -3
usemtl none
f 1//1 3//1 5//1
f 2/2 3/3 5/1
""",
}
for k, v in files.items():
    with open(os.path.join(out, k), "wb") as f:
        f.write(v)
print(" ".join(sorted(files)))
