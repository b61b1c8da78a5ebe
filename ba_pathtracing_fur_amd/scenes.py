"""Flattened scenes and the seeded synthetic inputs of BASELINE.json's configs.

A `SceneData` is what KIRK's CPU::Scene::flattenNode produces before the
Triangle/Cylinder constructors run (CPU_Scene.cpp:73-197): world-space
triangles, cone frusta (from fur fibers, CPU_Scene.cpp:121-144), materials,
lights, environment and camera.  It is plain data: the same arrays feed the
HIP core (product) and, in tests, the CPU restatement under oracle/.

Geometry generators run in libkirk_hip.so's host code (khp_gen_*), so the
inputs are bit-identical on every host.  Cornell-box / plane vertices are
exact constants.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import native as N

SEED = 0x4B49524B  # "KIRK" 

FIBER_DIFFUSE = (0.545, 0.353, 0.169)  # CPU_Scene.cpp:116
FIBER_IOR = 1.55                       # CPU_Scene.cpp:117


def material(bsdf="LambertianReflectionBSDF", shader=None, diffuse=(1, 1, 1), specular=(1, 1, 1),
             volume=(1, 1, 1), emission=(0, 0, 0), ior=1.52, roughness=1.0) -> N.Material:
    """KIRK::Material defaults (Material.h:69-83): white colours, ior 1.52, roughness 1."""
    if bsdf not in N.BSDF_NAMES:
        raise ValueError(f"BSDF {bsdf!r} is not registered")  # BsdfFactory.cpp:39-45 throws invalid_argument
    if shader is None:
        shader = "MarschnerHairShader" if bsdf in ("MarschnerHairBSDF", "DEonHairBSDF") else "SimpleShader"
    if shader not in N.SHADER_NAMES:
        raise ValueError(f"shader {shader!r} is not registered")
    m = N.Material()
    m.bsdf = N.BSDF_NAMES.index(bsdf)
    m.shader = N.SHADER_NAMES.index(shader)
    m.diffuse[:] = diffuse
    m.specular[:] = specular
    m.volume[:] = volume
    m.emission[:] = emission
    m.ior = ior
    m.roughness = roughness
    return m


def fiber_material(bsdf="MarschnerHairBSDF") -> N.Material:
    """Material("Fiber_Mat", true) as CPU_Scene.cpp:115-118 builds it."""
    return material(bsdf, "MarschnerHairShader", diffuse=FIBER_DIFFUSE, ior=FIBER_IOR)


def quad_light(position, direction, size, color, att_const=0.0, att_lin=0.0, att_quad=0.001) -> N.Light:
    """QuadLight ctor args (Light.h QuadLight defaults: const 0, lin 0, quad 0.001)."""
    L = N.Light()
    L.kind = N.LIGHT_QUAD
    L.position[:] = position
    L.direction[:] = direction
    L.size[:] = size
    L.color[:] = color
    L.att_const, L.att_lin, L.att_quad = att_const, att_lin, att_quad
    return L


def point_light(position, color, radius=0.8, att_const=1.0, att_lin=0.0, att_quad=0.001) -> N.Light:
    L = N.Light()
    L.kind = N.LIGHT_POINT
    L.position[:] = position
    L.color[:] = color
    L.radius = radius
    L.att_const, L.att_lin, L.att_quad = att_const, att_lin, att_quad
    return L


def spot_light(position, direction, color, radius=0.5, outer=22.5, inner=-1.0, att_const=0.0, att_lin=0.0,
               att_quad=0.0) -> N.Light:
    L = N.Light()
    L.kind = N.LIGHT_SPOT
    L.position[:] = position
    L.direction[:] = direction
    L.color[:] = color
    L.radius = radius
    L.outer_angle, L.inner_angle = outer, inner
    L.att_const, L.att_lin, L.att_quad = att_const, att_lin, att_quad
    return L


def sun_light(direction, color, radius=0.01) -> N.Light:
    L = N.Light()
    L.kind = N.LIGHT_SUN
    L.direction[:] = direction
    L.color[:] = color
    L.radius = radius
    return L


def camera(position, look_at, up=(0.0, 1.0, 0.0), width=256, height=256, sensor=(0.036, 0.024),
           focal=0.0415) -> N.Camera:
    """Camera::applyParameters (Camera.cpp:6-37) via khp_camera_setup."""
    lib = N.load_library()
    cam = N.Camera()
    p = np.asarray(position, np.float32)
    la = np.asarray(look_at, np.float32)
    u = np.asarray(up, np.float32)
    N.check(lib, lib.khp_camera_setup(N.fptr(p), N.fptr(la), N.fptr(u), sensor[0], sensor[1], focal, width, height,
                                      ctypes.byref(cam)), "khp_camera_setup")
    return cam


@dataclass
class SceneData:
    tri_v: np.ndarray = field(default_factory=lambda: np.zeros((0, 3, 3), np.float32))
    tri_n: np.ndarray = field(default_factory=lambda: np.zeros((0, 3, 3), np.float32))
    tri_mat: np.ndarray = field(default_factory=lambda: np.zeros((0,), np.uint32))
    # hair frame (u, v, w) per triangle: set by fiberToTriangles fur, zero otherwise
    tri_frame: np.ndarray = field(default_factory=lambda: np.zeros((0, 3, 3), np.float32))
    cone_base_r0: np.ndarray = field(default_factory=lambda: np.zeros((0, 4), np.float32))
    cone_apex_r1: np.ndarray = field(default_factory=lambda: np.zeros((0, 4), np.float32))
    cone_mat: np.ndarray = field(default_factory=lambda: np.zeros((0,), np.uint32))
    materials: list = field(default_factory=list)
    lights: list = field(default_factory=list)
    env_color: tuple = (0.0, 0.0, 0.0)
    env_ambient: tuple = (0.1, 0.1, 0.1)  # Environment.h:158 default
    cam: N.Camera | None = None
    name: str = "scene"

    # --- building ------------------------------------------------------------
    def add_material(self, m: N.Material) -> int:
        self.materials.append(m)
        return len(self.materials) - 1

    def add_triangles(self, v: np.ndarray, n: np.ndarray, mat: int, frame: np.ndarray | None = None):
        """Triangles (a, b, c) with vertex normals; frame: optional hair frame u, v, w per
        triangle (Object::setU/V/W, fiberToTriangles fur), zero otherwise."""
        v = np.ascontiguousarray(v, np.float32).reshape(-1, 3, 3)
        n = np.ascontiguousarray(n, np.float32).reshape(-1, 3, 3)
        old = self.frames()
        self.tri_v = np.concatenate([self.tri_v, v])
        self.tri_n = np.concatenate([self.tri_n, n])
        self.tri_mat = np.concatenate([self.tri_mat, np.full(len(v), mat, np.uint32)])
        f = np.zeros((len(v), 3, 3), np.float32) if frame is None else np.asarray(frame, np.float32).reshape(-1, 3, 3)
        self.tri_frame = np.concatenate([old, f])

    def frames(self) -> np.ndarray:
        """tri_frame padded with zero frames to one per triangle."""
        f = np.asarray(self.tri_frame, np.float32).reshape(-1, 3, 3)
        if len(f) < len(self.tri_v):
            f = np.concatenate([f, np.zeros((len(self.tri_v) - len(f), 3, 3), np.float32)])
        return f

    def add_fibers(self, positions: np.ndarray, radii: np.ndarray, mat: int, as_triangles: bool = False,
                   resolution: int = 5):
        """Fur fibers -> cones exactly as CPU_Scene::flattenNode (khp_fibers_to_cones), or, with
        as_triangles (m_fiberAsCylinder = false), -> triangle tubes as fiberToTriangles
        (khp_fibers_to_triangles, CPU_Scene.cpp:232-345)."""
        lib = N.load_library()
        positions = np.ascontiguousarray(positions, np.float32)
        radii = np.ascontiguousarray(radii, np.float32)
        nf, nv = radii.shape
        if as_triangles:
            nt = nf * (nv - 1) * 2 * resolution * resolution
            v = np.empty((nt, 3, 3), np.float32)
            n = np.empty((nt, 3, 3), np.float32)
            fr = np.empty((nt, 3, 3), np.float32)
            N.check(lib, lib.khp_fibers_to_triangles(nf, nv, N.fptr(positions), N.fptr(radii), resolution, N.fptr(v),
                                                     N.fptr(n), N.fptr(fr)), "khp_fibers_to_triangles")
            self.add_triangles(v, n, mat, frame=fr)
            return
        base = np.empty((nf * (nv - 1), 4), np.float32)
        apex = np.empty((nf * (nv - 1), 4), np.float32)
        N.check(lib, lib.khp_fibers_to_cones(nf, nv, N.fptr(positions), N.fptr(radii), N.fptr(base), N.fptr(apex)),
                "khp_fibers_to_cones")
        self.add_cones(base, apex, mat)

    def add_cones(self, base_r0: np.ndarray, apex_r1: np.ndarray, mat: int):
        self.cone_base_r0 = np.concatenate([self.cone_base_r0, np.asarray(base_r0, np.float32).reshape(-1, 4)])
        self.cone_apex_r1 = np.concatenate([self.cone_apex_r1, np.asarray(apex_r1, np.float32).reshape(-1, 4)])
        self.cone_mat = np.concatenate([self.cone_mat, np.full(len(base_r0), mat, np.uint32)])

    @property
    def n_objects(self) -> int:
        return len(self.tri_v) + len(self.cone_base_r0)

    # --- boundary struct ---------------------------------------------------------
    def desc(self) -> N.SceneDesc:
        """khp_scene view; arrays stay owned by this object (keep it alive)."""
        self.tri_v = np.ascontiguousarray(self.tri_v, np.float32)
        self.tri_n = np.ascontiguousarray(self.tri_n, np.float32)
        self.tri_mat = np.ascontiguousarray(self.tri_mat, np.uint32)
        self.tri_frame = np.ascontiguousarray(self.frames(), np.float32)
        self.cone_base_r0 = np.ascontiguousarray(self.cone_base_r0, np.float32)
        self.cone_apex_r1 = np.ascontiguousarray(self.cone_apex_r1, np.float32)
        self.cone_mat = np.ascontiguousarray(self.cone_mat, np.uint32)
        self._mats = (N.Material * max(1, len(self.materials)))(*self.materials)
        self._lights = (N.Light * max(1, len(self.lights)))(*self.lights)
        d = N.SceneDesc()
        d.n_tris = len(self.tri_v)
        d.tri_v = N.fptr(self.tri_v)
        d.tri_n = N.fptr(self.tri_n)
        d.tri_mat = N.uptr(self.tri_mat)
        d.tri_frame = N.fptr(self.tri_frame)
        d.n_cones = len(self.cone_base_r0)
        d.cone_base_r0 = N.fptr(self.cone_base_r0)
        d.cone_apex_r1 = N.fptr(self.cone_apex_r1)
        d.cone_mat = N.uptr(self.cone_mat)
        d.n_materials = len(self.materials)
        d.materials = ctypes.cast(self._mats, ctypes.POINTER(N.Material))
        d.n_lights = len(self.lights)
        d.lights = ctypes.cast(self._lights, ctypes.POINTER(N.Light))
        d.env.color[:] = self.env_color
        d.env.ambient[:] = self.env_ambient
        if self.cam is None:
            raise ValueError("scene has no camera")
        d.camera = self.cam
        self._desc = d
        return d

    # --- plain-data (de)serialisation: .npz of arrays + raw boundary structs -----------
    def to_arrays(self) -> dict:
        """Arrays for np.savez; materials/lights/camera are their khp_* struct bytes."""
        raw = lambda objs, T: np.frombuffer(bytes((T * len(objs))(*objs)), np.uint8).copy()
        return {"tri_v": self.tri_v, "tri_n": self.tri_n, "tri_mat": self.tri_mat, "tri_frame": self.frames(),
                "cone_base_r0": self.cone_base_r0, "cone_apex_r1": self.cone_apex_r1, "cone_mat": self.cone_mat,
                "materials": raw(self.materials, N.Material), "lights": raw(self.lights, N.Light),
                "env": np.float32([*self.env_color, *self.env_ambient]),
                "camera": np.frombuffer(bytes(self.cam), np.uint8).copy(), "name": np.array(self.name)}

    @classmethod
    def from_arrays(cls, a) -> "SceneData":
        def structs(buf, T):
            buf = np.ascontiguousarray(buf, np.uint8).tobytes()
            n = len(buf) // ctypes.sizeof(T)
            return list((T * n).from_buffer_copy(buf)) if n else []
        env = np.asarray(a["env"], np.float32)
        return cls(tri_v=np.asarray(a["tri_v"], np.float32), tri_n=np.asarray(a["tri_n"], np.float32),
                   tri_mat=np.asarray(a["tri_mat"], np.uint32),
                   tri_frame=np.asarray(a["tri_frame"], np.float32) if "tri_frame" in getattr(a, "files", a)
                   else np.zeros((0, 3, 3), np.float32),
                   cone_base_r0=np.asarray(a["cone_base_r0"], np.float32),
                   cone_apex_r1=np.asarray(a["cone_apex_r1"], np.float32),
                   cone_mat=np.asarray(a["cone_mat"], np.uint32),
                   materials=structs(a["materials"], N.Material), lights=structs(a["lights"], N.Light),
                   env_color=tuple(float(x) for x in env[:3]), env_ambient=tuple(float(x) for x in env[3:]),
                   cam=N.Camera.from_buffer_copy(np.ascontiguousarray(a["camera"], np.uint8).tobytes()),
                   name=str(a["name"]))


# ---- generators (libkirk_hip host code) -------------------------------------------
def hairball(n_strands: int, center, ball_radius: float, root_radius: float = 0.004, verts: int = 10,
             seed: int = SEED):
    """Seeded hairball: addFurToFaces recurrence (Mesh.cpp:118-142) on sphere roots."""
    lib = N.load_library()
    pos = np.empty((n_strands, verts, 3), np.float32)
    rad = np.empty((n_strands, verts), np.float32)
    c = np.asarray(center, np.float32)
    N.check(lib, lib.khp_gen_hairball(n_strands, verts, N.fptr(c), ball_radius, root_radius, seed, N.fptr(pos),
                                      N.fptr(rad)), "khp_gen_hairball")
    return pos, rad


def icosphere(subdiv: int, center, radius: float):
    lib = N.load_library()
    n = 20 * 4 ** subdiv
    v = np.empty((n, 3, 3), np.float32)
    nn = np.empty((n, 3, 3), np.float32)
    c = np.asarray(center, np.float32)
    N.check(lib, lib.khp_gen_icosphere(subdiv, N.fptr(c), radius, N.fptr(v), N.fptr(nn)), "khp_gen_icosphere")
    return v, nn


def torus(nu: int, nv: int, center, major: float, minor: float):
    lib = N.load_library()
    n = 2 * nu * nv
    v = np.empty((n, 3, 3), np.float32)
    nn = np.empty((n, 3, 3), np.float32)
    c = np.asarray(center, np.float32)
    N.check(lib, lib.khp_gen_torus(nu, nv, N.fptr(c), major, minor, N.fptr(v), N.fptr(nn)), "khp_gen_torus")
    return v, nn


def quad(p0, p1, p2, p3, normal):
    """Two triangles (p0,p1,p2), (p0,p2,p3) with a constant vertex normal."""
    v = np.array([[p0, p1, p2], [p0, p2, p3]], np.float32)
    n = np.broadcast_to(np.asarray(normal, np.float32), (2, 3, 3)).copy()
    return v, n


# ---- BASELINE.json configs ------------------------------------------
def cornell_box(sd: SceneData, width: int, height: int):
    """Unit Cornell box x,z in [-0.5,0.5], y in [0,1], open towards +z, quad light in the ceiling."""
    white = sd.add_material(material(diffuse=(0.725, 0.725, 0.725)))
    red = sd.add_material(material(diffuse=(0.63, 0.065, 0.05)))
    green = sd.add_material(material(diffuse=(0.14, 0.45, 0.091)))
    a, b = -0.5, 0.5
    for (v, n), m in [
        (quad((a, 0, a), (b, 0, a), (b, 0, b), (a, 0, b), (0, 1, 0)), white),      # floor
        (quad((a, 1, a), (a, 1, b), (b, 1, b), (b, 1, a), (0, -1, 0)), white),     # ceiling
        (quad((a, 0, a), (a, 1, a), (b, 1, a), (b, 0, a), (0, 0, 1)), white),      # back
        (quad((a, 0, a), (a, 0, b), (a, 1, b), (a, 1, a), (1, 0, 0)), red),        # left
        (quad((b, 0, a), (b, 1, a), (b, 1, b), (b, 0, b), (-1, 0, 0)), green),     # right
    ]:
        sd.add_triangles(v, n, m)
    sd.lights.append(quad_light((0.0, 0.999, 0.0), (0.0, -1.0, 0.0), (0.25, 0.25), (17.0, 12.0, 4.0),
                                att_const=1.0, att_lin=0.0, att_quad=0.0))
    sd.env_color = (0.0, 0.0, 0.0)
    sd.env_ambient = (0.0, 0.0, 0.0)
    sd.cam = camera((0.0, 0.5, 1.85), (0.0, 0.0, -1.0), (0.0, 1.0, 0.0), width, height)


def config1(width=256, height=256) -> SceneData:
    """Cornell box + 1 Lambert icosphere (subdiv 4, 5,120 tris, r=0.3)."""
    sd = SceneData(name="cornell_sphere")
    cornell_box(sd, width, height)
    v, n = icosphere(4, (0.0, 0.3, 0.0), 0.3)
    sd.add_triangles(v, n, sd.add_material(material(diffuse=(0.725, 0.725, 0.725))))
    return sd


def config2(width=1920, height=1080, n_strands=10_000, bsdf="MarschnerHairBSDF") -> SceneData:
    """Cornell box + procedural hairball (r=0.25, centre of the box), fur BSDF."""
    sd = SceneData(name=f"cornell_hairball_{n_strands}")
    cornell_box(sd, width, height)
    pos, rad = hairball(n_strands, (0.0, 0.5, 0.0), 0.25)
    sd.add_fibers(pos, rad, sd.add_material(fiber_material(bsdf)))
    return sd


def config3(width=1920, height=1080, n_strands=1_000_000, bsdf="MarschnerHairBSDF") -> SceneData:
    """Hairball (r=1.0) on a 2-tri diffuse plane + 2x2 area light at height 3, sky environment."""
    sd = SceneData(name=f"plane_hairball_{n_strands}")
    grey = sd.add_material(material(diffuse=(0.5, 0.5, 0.5)))
    v, n = quad((-6, 0, -6), (-6, 0, 6), (6, 0, 6), (6, 0, -6), (0, 1, 0))
    sd.add_triangles(v, n, grey)
    pos, rad = hairball(n_strands, (0.0, 1.0, 0.0), 1.0)
    sd.add_fibers(pos, rad, sd.add_material(fiber_material(bsdf)))
    sd.lights.append(quad_light((0.0, 3.0, 0.0), (0.0, -1.0, 0.0), (2.0, 2.0), (5.0, 5.0, 5.0),
                                att_const=1.0, att_lin=0.0, att_quad=0.0))
    sd.env_color = (0.7, 0.9, 1.0)
    sd.env_ambient = (0.1, 0.1, 0.1)
    sd.cam = camera((0.0, 1.4, 4.6), (0.0, -0.12, -1.0), (0.0, 1.0, 0.0), width, height)
    return sd


def config3_device(ctx, width=1920, height=1080, n_strands=1_000_000, bsdf="MarschnerHairBSDF") -> SceneData:
    """config3 with the hairball generated and flattened on the GPU of `ctx`
    (khp_gen_hairball_device + khp_set_scene_device).  The same
    objects in the same order as config3, so the same tree and frames.  Returns
    the host part (plane, materials, lights, camera); the cones live in HBM."""
    sd = config3(width, height, 0, bsdf)
    sd.name = f"plane_hairball_{n_strands}_device"
    base, apex, nc = ctx.hairball_device(n_strands, (0.0, 1.0, 0.0), 1.0)
    ctx.set_scene_device(sd, cones=(base, apex, nc, 1))
    base.free()
    apex.free()
    return sd


def config5(width=3840, height=2160, n_strands=1_000_000, torus_grid=500, glass_subdiv=5) -> SceneData:
    """Config 3 hairball + 500k-tri Lambert torus + glass icosphere (ior 1.52)."""
    sd = config3(width, height, n_strands)
    sd.name = f"mixed_{n_strands}"
    tv, tn = torus(torus_grid, torus_grid, (2.4, 0.45, -0.8), 0.8, 0.3)
    sd.add_triangles(tv, tn, sd.add_material(material(diffuse=(0.2, 0.4, 0.8))))
    gv, gn = icosphere(glass_subdiv, (-2.2, 0.7, 0.3), 0.7)
    sd.add_triangles(gv, gn, sd.add_material(material("GlassBSDF", ior=1.52)))
    return sd


def config5_device(ctx, width=3840, height=2160, n_strands=1_000_000, torus_grid=500,
                   glass_subdiv=5) -> SceneData:
    """config5 with the hairball generated and flattened on the GPU of `ctx`
    (as config3_device); the torus and the glass sphere come from the host.
    The same objects in the same order as config5 (triangles, then cones)."""
    sd = config5(width, height, 0, torus_grid, glass_subdiv)
    sd.name = f"mixed_{n_strands}_device"
    base, apex, nc = ctx.hairball_device(n_strands, (0.0, 1.0, 0.0), 1.0)
    ctx.set_scene_device(sd, cones=(base, apex, nc, 1))
    base.free()
    apex.free()
    return sd


def zoo(width=64, height=48, n_strands=400) -> SceneData:
    """Every BSDF of the zoo (Bsdf.cpp) and every light kind (Light.cpp) in one frame.

    Not a BASELINE config: a coverage scene for parity tests.  A row of small
    icospheres carries the nine surface BSDFs, two hairballs carry the Marschner
    and d'Eon fibers; point, quad, spot and sun lights all contribute.
    """
    sd = SceneData(name="zoo")
    v, n = quad((-4, 0, -4), (-4, 0, 4), (4, 0, 4), (4, 0, -4), (0, 1, 0))
    sd.add_triangles(v, n, sd.add_material(material(diffuse=(0.6, 0.6, 0.6))))
    v, n = quad((-4, 0, -2.5), (4, 0, -2.5), (4, 3, -2.5), (-4, 3, -2.5), (0, 0, 1))
    sd.add_triangles(v, n, sd.add_material(material(diffuse=(0.3, 0.5, 0.3))))
    surf = [material("LambertianReflectionBSDF", diffuse=(0.8, 0.3, 0.2)),
            material("SpecularReflectionBSDF", specular=(0.9, 0.9, 0.7)),
            material("SpecularTransmissionBSDF", volume=(0.9, 1.0, 0.9), ior=1.33),
            material("GlossyBSDF", diffuse=(0.2, 0.3, 0.8), specular=(0.8, 0.8, 0.8), roughness=0.3),
            material("GlassBSDF", volume=(1.0, 0.95, 0.9), ior=1.52),
            material("MilkGlassBSDF", diffuse=(0.9, 0.9, 0.9), volume=(0.9, 0.9, 1.0), ior=1.45, roughness=0.5),
            material("LambertianTransmissionBSDF", diffuse=(0.7, 0.7, 0.2)),
            material("EmissionBSDF", emission=(2.0, 1.0, 0.5)),
            material("TransparentBSDF", volume=(0.5, 0.8, 1.0))]
    for i, m in enumerate(surf):
        gv, gn = icosphere(1, (-2.4 + 0.6 * i, 0.3, -0.6 + 0.35 * (i % 2)), 0.27)
        sd.add_triangles(gv, gn, sd.add_material(m))
    for k, bsdf in enumerate(("MarschnerHairBSDF", "DEonHairBSDF")):
        pos, rad = hairball(n_strands, (-0.9 + 1.8 * k, 0.9, 0.8), 0.3, root_radius=0.006, seed=SEED + k)
        sd.add_fibers(pos, rad, sd.add_material(fiber_material(bsdf)))
    sd.lights += [point_light((1.5, 2.5, 1.5), (4.0, 3.5, 3.0), radius=0.2),
                  quad_light((0.0, 2.8, 0.0), (0.0, -1.0, 0.0), (1.0, 1.0), (3.0, 3.0, 3.0), att_const=1.0),
                  spot_light((-2.0, 2.5, 1.0), (0.5, -1.0, -0.3), (6.0, 5.0, 4.0), outer=30.0, inner=15.0,
                             att_const=1.0),
                  sun_light((0.3, -1.0, -0.4), (0.8, 0.8, 0.7))]
    sd.env_color = (0.2, 0.25, 0.35)
    sd.env_ambient = (0.05, 0.05, 0.05)
    sd.cam = camera((0.0, 1.5, 4.2), (0.0, -0.25, -1.0), (0.0, 1.0, 0.0), width, height)
    return sd


def build_config(name: str, **kw) -> SceneData:
    return {"config1": config1, "config2": config2, "config3": config3, "config5": config5, "zoo": zoo}[name](**kw)
