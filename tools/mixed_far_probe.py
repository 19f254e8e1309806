import sys, json, time, os
sys.path.insert(0, os.getcwd())
import numpy as np
from ptsharp_amd import Renderer, _abi, scenes, Matrix, Vector, TransformedShape, SDFShape, TransformSDF, TorusSDF, Material, Colour, Util
from ptsharp_amd.scenes import F
def build(far):
    scene, camera, sampler = scenes.bunny_frame(1_000_000, seed=1234)
    scene.Texture = scenes.seeded_texture(512, 256, 21)
    scene.TextureAngle = Util.Radians(40)
    off = Vector(0, 200, 0) if far else Vector(0, 0, 0)
    ring = TransformSDF.NewTransformSDF(TorusSDF.NewTorusSDF(F(0.45), F(0.12)),
                                        Matrix.TranslateM(Vector(-1.8, 0.5, 0.4).Add(off)).Mul(Matrix.RotateM(Vector(1, 0, 0), Util.Radians(70))))
    scene.Add(SDFShape.NewSDFShape(ring, Material.GlossyMaterial(Colour.HexColor(0x1F8A70), F(1.4), Util.Radians(10))))
    vol, _, _ = scenes.volume(32, 32, 16, seed=5)
    scene.Add(TransformedShape.NewTransformedShape(vol.Shapes[0], Matrix.TranslateM(Vector(1.6, 0.55, -0.6).Add(off)).Mul(Matrix.ScaleM(Vector(0.5, 0.5, 0.5)))))
    return scene, camera, sampler
for far in (False, True, None):
    if far is None:
        scene, camera, sampler = scenes.bunny_frame(1_000_000, seed=1234)
        scene.Texture = scenes.seeded_texture(512, 256, 21)
    else:
        scene, camera, sampler = build(far)
    r = Renderer.NewRenderer(scene, camera, sampler, 3840, 2160, True)
    r.SamplesPerPixel = 1; r.Seed = 1234; r.Engine = _abi.ENGINE_WAVEFRONT
    r.RenderParallel(); r.Flags = _abi.PASS_KERNEL_TIMING; r.Synchronize()
    t0 = time.perf_counter(); rays = 0; kms = np.zeros(_abi.K_SLOTS)
    for _ in range(2):
        r.RenderParallel(); st = r.Stats(); rays += st.rays; kms += np.array(st.kernel_ms[:])
    r.Synchronize(); dt = time.perf_counter() - t0
    print(json.dumps({"far": far, "Mrays": round(rays/dt/1e6,1), "trace": round(kms[1]/2,1), "shade": round(kms[2]/2,1), "shadow": round(kms[3]/2,1)}), flush=True)
    r.close()
