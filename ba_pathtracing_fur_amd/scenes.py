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
    # ABI 6: cone node transforms (glm::mat4, column-major) and per-cone model index
    cone_models: np.ndarray = field(default_factory=lambda: np.zeros((0, 16), np.float32))
    cone_model: np.ndarray = field(default_factory=lambda: np.zeros((0,), np.uint32))
    # ABI 6: textures [(texels (H, W, C) uint8, wrap_mode)], per-material texture ids (n_mat, 5)
    # (diffuse, specular, volume, emission, roughness; -1 = value), texcoords, environment map
    textures: list = field(default_factory=list)
    material_textures: np.ndarray | None = None
    tri_uv: np.ndarray = field(default_factory=lambda: np.zeros((0, 3, 2), np.float32))
    env_map: tuple = (0, (-1, -1, -1, -1, -1, -1))

    # --- building ------------------------------------------------------------
    def add_material(self, m: N.Material) -> int:
        self.materials.append(m)
        return len(self.materials) - 1

    def add_triangles(self, v: np.ndarray, n: np.ndarray, mat: int, frame: np.ndarray | None = None,
                      uv: np.ndarray | None = None):
        """Triangles (a, b, c) with vertex normals; frame: optional hair frame u, v, w per
        triangle (Object::setU/V/W, fiberToTriangles fur), zero otherwise; uv: optional
        texcoords tca, tcb, tcc per triangle (zero otherwise)."""
        v = np.ascontiguousarray(v, np.float32).reshape(-1, 3, 3)
        n = np.ascontiguousarray(n, np.float32).reshape(-1, 3, 3)
        old_uv = self.uvs()
        self.tri_uv = np.concatenate([old_uv, np.zeros((len(v), 3, 2), np.float32) if uv is None
                                      else np.asarray(uv, np.float32).reshape(-1, 3, 2)])
        old = self.frames()
        self.tri_v = np.concatenate([self.tri_v, v])
        self.tri_n = np.concatenate([self.tri_n, n])
        self.tri_mat = np.concatenate([self.tri_mat, np.full(len(v), mat, np.uint32)])
        f = np.zeros((len(v), 3, 3), np.float32) if frame is None else np.asarray(frame, np.float32).reshape(-1, 3, 3)
        self.tri_frame = np.concatenate([old, f])

    def uvs(self) -> np.ndarray:
        """tri_uv padded with zero texcoords to one triple per triangle."""
        u = np.asarray(self.tri_uv, np.float32).reshape(-1, 3, 2)
        if len(u) < len(self.tri_v):
            u = np.concatenate([u, np.zeros((len(self.tri_v) - len(u), 3, 2), np.float32)])
        return u

    def add_texture(self, texels: np.ndarray, wrap_mode: int = N.TEX_WRAP_TILE) -> int:
        """A KIRK::Texture: (H, W, C) uint8, C in 1..4, row y = texture row y."""
        t = np.ascontiguousarray(texels, np.uint8)
        if t.ndim == 2:
            t = t[:, :, None]
        self.textures.append((t, int(wrap_mode)))
        return len(self.textures) - 1

    def set_material_texture(self, mat: int, param: str, tex: int):
        """Textures material parameter `param` (diffuse | specular | volume | emission | roughness)."""
        keys = ["diffuse", "specular", "volume", "emission", "roughness"]
        if self.material_textures is None or len(self.material_textures) < len(self.materials):
            mt = np.full((len(self.materials), 5), -1, np.int32)
            if self.material_textures is not None:
                mt[:len(self.material_textures)] = self.material_textures
            self.material_textures = mt
        self.material_textures[mat, keys.index(param)] = tex

    def set_environment_map(self, kind: int, tex):
        """Environment::loadCubeMap (6 textures: posx, posy, posz, negx, negy, negz) or loadSphereMap."""
        t = list(tex) + [-1] * (6 - len(tex))
        self.env_map = (int(kind), tuple(int(x) for x in t))

    def add_cone_model(self, M: np.ndarray) -> int:
        """A node transform (4x4, row-major numpy matrix acting on column vectors) for cones."""
        m = np.asarray(M, np.float32).reshape(4, 4)
        self.cone_models = np.concatenate([self.cone_models, m.T.reshape(1, 16)])  # glm: column-major
        return len(self.cone_models) - 1

    def frames(self) -> np.ndarray:
        """tri_frame padded with zero frames to one per triangle."""
        f = np.asarray(self.tri_frame, np.float32).reshape(-1, 3, 3)
        if len(f) < len(self.tri_v):
            f = np.concatenate([f, np.zeros((len(self.tri_v) - len(f), 3, 3), np.float32)])
        return f

    def add_fibers(self, positions: np.ndarray, radii: np.ndarray, mat: int, as_triangles: bool = False,
                   resolution: int = 5, model: int | None = None):
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
        self.add_cones(base, apex, mat, model)

    def add_cones(self, base_r0: np.ndarray, apex_r1: np.ndarray, mat: int, model: int | None = None):
        """Cones (Cylinder ctor args); model: index of a node transform (add_cone_model),
        None = world space (an identity model once any cone of the scene has one)."""
        n_old = len(self.cone_base_r0)
        self.cone_base_r0 = np.concatenate([self.cone_base_r0, np.asarray(base_r0, np.float32).reshape(-1, 4)])
        self.cone_apex_r1 = np.concatenate([self.cone_apex_r1, np.asarray(apex_r1, np.float32).reshape(-1, 4)])
        self.cone_mat = np.concatenate([self.cone_mat, np.full(len(base_r0), mat, np.uint32)])
        if model is None and len(self.cone_models) == 0:
            return
        if len(self.cone_model) < n_old:  # earlier world-space cones: the identity model
            ident = self.add_cone_model(np.eye(4))
            self.cone_model = np.concatenate([self.cone_model, np.full(n_old - len(self.cone_model), ident, np.uint32)])
        if model is None:
            model = self.add_cone_model(np.eye(4))
        self.cone_model = np.concatenate([self.cone_model, np.full(len(base_r0), model, np.uint32)])

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
        # ABI 6
        self.cone_models = np.ascontiguousarray(self.cone_models, np.float32).reshape(-1, 16)
        d.n_cone_models = len(self.cone_models)
        d.cone_models = N.fptr(self.cone_models)
        if len(self.cone_models):
            if len(self.cone_model) != len(self.cone_base_r0):
                raise ValueError("cone_model must name a model for every cone")
            self.cone_model = np.ascontiguousarray(self.cone_model, np.uint32)
            d.cone_model = N.uptr(self.cone_model)
        self._tex = [np.ascontiguousarray(t, np.uint8) for t, _ in self.textures]
        self._texs = (N.Texture * max(1, len(self.textures)))()
        for i, ((t, wrap), data) in enumerate(zip(self.textures, self._tex)):
            self._texs[i] = N.Texture(t.shape[1], t.shape[0], t.shape[2], wrap,
                                      data.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
        d.n_textures = len(self.textures)
        d.textures = ctypes.cast(self._texs, ctypes.POINTER(N.Texture))
        if self.material_textures is not None:
            mt = np.full((len(self.materials), 5), -1, np.int32)
            mt[:len(self.material_textures)] = self.material_textures
            self._mtex = (N.MaterialTextures * len(self.materials))(*[N.MaterialTextures(*map(int, r)) for r in mt])
            d.material_textures = ctypes.cast(self._mtex, ctypes.POINTER(N.MaterialTextures))
        if self.textures:
            self.tri_uv = np.ascontiguousarray(self.uvs(), np.float32)
            d.tri_uv = N.fptr(self.tri_uv)
        d.env_map.type = self.env_map[0]
        d.env_map.tex[:] = self.env_map[1]
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
                "camera": np.frombuffer(bytes(self.cam), np.uint8).copy(), "name": np.array(self.name),
                "cone_models": self.cone_models, "cone_model": self.cone_model, "tri_uv": self.uvs(),
                "material_textures": (np.zeros((0, 5), np.int32) if self.material_textures is None
                                      else self.material_textures),
                "env_map": np.int32([self.env_map[0], *self.env_map[1]]),
                "n_textures": np.int32(len(self.textures)),
                **{f"texture{i}": t for i, (t, _) in enumerate(self.textures)},
                "texture_wrap": np.int32([w for _, w in self.textures])}

    @classmethod
    def from_arrays(cls, a) -> "SceneData":
        def structs(buf, T):
            buf = np.ascontiguousarray(buf, np.uint8).tobytes()
            n = len(buf) // ctypes.sizeof(T)
            return list((T * n).from_buffer_copy(buf)) if n else []
        files = set(getattr(a, "files", a))
        get = lambda k, default: a[k] if k in files else default
        env = np.asarray(a["env"], np.float32)
        sd = cls(tri_v=np.asarray(a["tri_v"], np.float32), tri_n=np.asarray(a["tri_n"], np.float32),
                 tri_mat=np.asarray(a["tri_mat"], np.uint32),
                 tri_frame=np.asarray(get("tri_frame", np.zeros((0, 3, 3), np.float32)), np.float32),
                 cone_base_r0=np.asarray(a["cone_base_r0"], np.float32),
                 cone_apex_r1=np.asarray(a["cone_apex_r1"], np.float32),
                 cone_mat=np.asarray(a["cone_mat"], np.uint32),
                 materials=structs(a["materials"], N.Material), lights=structs(a["lights"], N.Light),
                 env_color=tuple(float(x) for x in env[:3]), env_ambient=tuple(float(x) for x in env[3:]),
                 cam=N.Camera.from_buffer_copy(np.ascontiguousarray(a["camera"], np.uint8).tobytes()),
                 name=str(a["name"]))
        sd.cone_models = np.asarray(get("cone_models", np.zeros((0, 16), np.float32)), np.float32).reshape(-1, 16)
        sd.cone_model = np.asarray(get("cone_model", np.zeros((0,), np.uint32)), np.uint32)
        sd.tri_uv = np.asarray(get("tri_uv", np.zeros((0, 3, 2), np.float32)), np.float32)
        mt = np.asarray(get("material_textures", np.zeros((0, 5), np.int32)), np.int32)
        sd.material_textures = mt if len(mt) else None
        em = np.asarray(get("env_map", np.int32([0, -1, -1, -1, -1, -1, -1])), np.int32)
        sd.env_map = (int(em[0]), tuple(int(x) for x in em[1:7]))
        wraps = np.asarray(get("texture_wrap", np.zeros((0,), np.int32)), np.int32)
        sd.textures = [(np.asarray(a[f"texture{i}"], np.uint8), int(wraps[i]))
                       for i in range(int(get("n_textures", 0)))]
        return sd


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


def checker(h: int, w: int, channels: int, cells: int = 4, seed: int = 7) -> np.ndarray:
    """Seeded checkerboard texels (H, W, C) uint8: `cells` x `cells` blocks of random colours."""
    rng = np.random.default_rng(seed)
    cols = rng.integers(0, 256, (cells, cells, channels), dtype=np.uint8)
    yy = (np.arange(h) * cells // h)[:, None]
    xx = (np.arange(w) * cells // w)[None, :]
    return np.ascontiguousarray(cols[yy, xx])


def rotation(axis, angle_rad: float) -> np.ndarray:
    a = np.asarray(axis, np.float64)
    a /= np.linalg.norm(a)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    R = np.eye(3) + np.sin(angle_rad) * K + (1 - np.cos(angle_rad)) * K @ K
    M = np.eye(4)
    M[:3, :3] = R
    return M


def node_transform(translate=(0, 0, 0), axis=(0, 1, 0), angle_rad=0.0, scale=(1, 1, 1)) -> np.ndarray:
    """T * R * S as a scene node's model matrix (float32)."""
    T = np.eye(4)
    T[:3, 3] = translate
    S = np.diag([*scale, 1.0])
    return (T @ rotation(axis, angle_rad) @ S).astype(np.float32)


def transformed_hairball(width=64, height=48, n_strands=1500, bsdf="MarschnerHairBSDF") -> SceneData:
    """Coverage scene for the Cylinder node transform (Cylinder.cpp:5-29): two
    hairball nodes in object space, one rotated about a tilted axis and scaled
    non-uniformly, one translated only, on a plane under a quad light."""
    sd = SceneData(name="transformed_hairball")
    v, n = quad((-6, 0, -6), (-6, 0, 6), (6, 0, 6), (6, 0, -6), (0, 1, 0))
    sd.add_triangles(v, n, sd.add_material(material(diffuse=(0.5, 0.5, 0.5))))
    fur = sd.add_material(fiber_material(bsdf))
    pos, rad = hairball(n_strands, (0.0, 0.0, 0.0), 0.35)
    m0 = sd.add_cone_model(node_transform((-0.45, 0.55, 0.0), (0.3, 1.0, 0.2), 0.7, (1.3, 0.8, 1.1)))
    sd.add_fibers(pos, rad, fur, model=m0)
    m1 = sd.add_cone_model(node_transform((0.5, 0.45, 0.1)))
    pos2, rad2 = hairball(n_strands // 2, (0.0, 0.0, 0.0), 0.3, seed=SEED + 1)
    sd.add_fibers(pos2, rad2, fur, model=m1)
    sd.lights.append(quad_light((0.0, 3.0, 0.0), (0.0, -1.0, 0.0), (2.0, 2.0), (5.0, 5.0, 5.0), att_const=1.0))
    sd.env_color = (0.6, 0.7, 0.9)
    sd.cam = camera((0.0, 0.8, 2.6), (0.0, -0.15, -1.0), (0.0, 1.0, 0.0), width, height)
    return sd


def textured(width=64, height=48, n_strands=600, env: str = "cube") -> SceneData:
    """Coverage scene for textures (Texture::getColor, Material::getFromParam,
    calcTcoord of triangles and cones, Environment cube / sphere maps): a
    diffuse-textured floor (tiled uv beyond [0, 1]), a glossy panel with
    textured specular + roughness, an emission-textured quad, a glass sphere
    with a textured volume colour, fur with a textured diffuse colour, and
    an environment map."""
    sd = SceneData(name=f"textured_{env}")
    t_floor = sd.add_texture(checker(32, 48, 3, 6, seed=1))
    t_spec = sd.add_texture(checker(16, 16, 4, 4, seed=2), N.TEX_WRAP_CLAMP)
    t_rough = sd.add_texture(checker(8, 8, 1, 2, seed=3))
    t_emit = sd.add_texture(checker(24, 24, 2, 3, seed=4))
    t_fur = sd.add_texture(checker(16, 64, 3, 8, seed=5))
    t_vol = sd.add_texture(checker(8, 8, 3, 2, seed=6))
    floor = sd.add_material(material(diffuse=(0.5, 0.5, 0.5)))
    sd.set_material_texture(floor, "diffuse", t_floor)
    v, n = quad((-4, 0, -4), (-4, 0, 4), (4, 0, 4), (4, 0, -4), (0, 1, 0))
    sd.add_triangles(v, n, floor, uv=np.float32([[[-1.5, -1.5], [-1.5, 2.5], [2.5, 2.5]],
                                                 [[-1.5, -1.5], [2.5, 2.5], [2.5, -1.5]]]))
    glossy = sd.add_material(material("GlossyBSDF", diffuse=(0.2, 0.3, 0.6), roughness=0.4))
    sd.set_material_texture(glossy, "specular", t_spec)
    sd.set_material_texture(glossy, "roughness", t_rough)
    v, n = quad((-1.8, 0, -1.5), (0.2, 0, -1.5), (0.2, 1.6, -1.5), (-1.8, 1.6, -1.5), (0, 0, 1))
    sd.add_triangles(v, n, glossy, uv=np.float32([[[0, 0], [1, 0], [1, 1]], [[0, 0], [1, 1], [0, 1]]]))
    emit = sd.add_material(material("EmissionBSDF", emission=(1.0, 1.0, 1.0)))
    sd.set_material_texture(emit, "emission", t_emit)
    v, n = quad((0.6, 0.2, -1.4), (1.8, 0.2, -1.4), (1.8, 1.4, -1.4), (0.6, 1.4, -1.4), (0, 0, 1))
    sd.add_triangles(v, n, emit, uv=np.float32([[[0, 0], [1, 0], [1, 1]], [[0, 0], [1, 1], [0, 1]]]))
    glass = sd.add_material(material("GlassBSDF", ior=1.45))
    sd.set_material_texture(glass, "volume", t_vol)
    gv, gn = icosphere(2, (1.3, 0.35, 0.3), 0.35)
    uv = np.stack([0.5 + 0.5 * np.arctan2(gv[..., 2] - 0.3, gv[..., 0] - 1.3) / np.pi, (gv[..., 1] - 0.0) / 0.7],
                  axis=-1).astype(np.float32)
    sd.add_triangles(gv, gn, glass, uv=uv)
    fur = sd.add_material(fiber_material())
    sd.set_material_texture(fur, "diffuse", t_fur)
    pos, rad = hairball(n_strands, (-0.3, 0.45, 0.2), 0.3, root_radius=0.006)
    sd.add_fibers(pos, rad, fur)
    sd.lights.append(quad_light((0.0, 2.8, 0.0), (0.0, -1.0, 0.0), (1.2, 1.2), (4.0, 4.0, 4.0), att_const=1.0))
    sd.lights.append(point_light((2.0, 2.0, 2.0), (2.0, 1.8, 1.5), radius=0.2))
    if env == "cube":
        faces = [sd.add_texture(checker(8, 8, 3, 2, seed=20 + k)) for k in range(6)]
        sd.set_environment_map(N.ENV_CUBE_MAP, faces)
    elif env == "sphere":
        sd.set_environment_map(N.ENV_SPHERE_MAP, [sd.add_texture(checker(32, 32, 3, 4, seed=30))])
    sd.env_ambient = (0.05, 0.05, 0.05)
    sd.cam = camera((0.0, 1.3, 3.4), (0.0, -0.25, -1.0), (0.0, 1.0, 0.0), width, height)
    return sd


def build_config(name: str, **kw) -> SceneData:
    return {"config1": config1, "config2": config2, "config3": config3, "config5": config5, "zoo": zoo,
            "transformed": transformed_hairball, "textured": textured}[name](**kw)
