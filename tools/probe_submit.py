import importlib, sys, time, os
sys.path.insert(0, os.getcwd())
rt = importlib.import_module("metal4-raytracing_amd")
sc = rt.Scene.preset("c3g")
R = rt.Renderer(sc, 1920, 1080, seed=3)
R.samplesPerPixel, R.maxBounces = 4, 8
for _ in range(3): R.draw()
R.wait()
# pure submission cost: draw with the GPU idle (slot free), then wait
ts = []
for _ in range(6):
    R.wait()
    t = time.perf_counter(); R.draw(); ts.append(time.perf_counter() - t)
R.wait()
print("submit ms (slot free):", [round(x * 1e3, 3) for x in ts])
u = R.uniforms()
ts = []
import ctypes as C
for _ in range(6):
    R.wait()
    t = time.perf_counter(); rt.lib().rt_render_frame(R._ctx, C.byref(u), None); ts.append(time.perf_counter() - t)
R.wait()
print("rt_render_frame ms:", [round(x * 1e3, 3) for x in ts])
