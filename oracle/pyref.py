"""pyref.py -- an independent pure-Python restatement of the reference render path.

TEST INFRASTRUCTURE ONLY (imported by tests/ to cross-check the C oracle).  Written directly
from the Rust sources of andreivasiliu/TinyRaytracerInRust, in the reference's own object
shape (classes with intersects / get_normal / is_inside / is_on_surface / get_uv_coordinates,
closures for CSG filters, recursive get_ray_color), independently of oracle/rt_oracle.c.
Python floats are IEEE-754 doubles evaluated left to right without contraction and `math`
calls the same glibc libm as Rust's f64 methods, so on small frames this must agree with the
C oracle BIT FOR BIT (tests/test_oracle.py).  Pure Python: keep frames tiny (<= 64x48).
"""
from __future__ import annotations

import math
import re

EPSILON = 10e-7                      # math.rs:2
PI = math.pi                         # std::f64::consts::PI
INF = math.inf


# ----------------------------------------------------------------------------- vector.rs
class Vector:
    __slots__ = ("x", "y", "z")

    def __init__(self, x, y, z):
        self.x, self.y, self.z = x, y, z

    def __add__(self, o):
        return Vector(self.x + o.x, self.y + o.y, self.z + o.z)

    def __sub__(self, o):
        return Vector(self.x - o.x, self.y - o.y, self.z - o.z)

    def dot(self, o):                 # impl Mul for Vector -> f64
        return self.x * o.x + self.y * o.y + self.z * o.z

    def scale(self, s):               # impl Mul<f64>
        return Vector(self.x * s, self.y * s, self.z * s)

    def __neg__(self):
        return Vector(-self.x, -self.y, -self.z)

    def length(self):
        return math.sqrt(self.dot(self))

    def normalized(self):
        return self.scale(div(1.0, self.length()))

    @staticmethod
    def angle(a, b):
        return acos(div(a.dot(b), a.length() * b.length()))

    @staticmethod
    def cross(a, b):
        return Vector(a.y * b.z - a.z * b.y, a.x * b.z - a.z * b.x, a.x * b.y - a.y * b.x)


def div(a, b):
    """IEEE f64 division (Python raises on /0; Rust gives +-inf or NaN)."""
    try:
        return a / b
    except ZeroDivisionError:
        if a != a or a == 0.0:
            return math.nan
        return math.copysign(math.inf, a) * math.copysign(1.0, b)


def acos(x):
    """f64::acos: NaN outside [-1, 1] (Python raises instead)."""
    if x != x or x > 1.0 or x < -1.0:
        return math.nan
    return math.acos(x)


def sin(x):
    if x != x or x in (INF, -INF):
        return math.nan
    return math.sin(x)


# ----------------------------------------------------------------------------- color.rs
def in_limit(x, lo, hi):
    if x < lo:
        return lo
    if x > hi:
        return hi
    return x


class Color:
    __slots__ = ("r", "g", "b", "a")

    def __init__(self, r, g, b, a=1.0):
        self.r, self.g, self.b, self.a = r, g, b, a

    @staticmethod
    def in_range(r, g, b):
        return Color(in_limit(r, 0.0, 1.0), in_limit(g, 0.0, 1.0), in_limit(b, 0.0, 1.0), 1.0)

    def intensify(self, k):
        return Color.in_range(self.r * k, self.g * k, self.b * k)

    def __mul__(self, o):
        return Color.in_range(self.r * o.r, self.g * o.g, self.b * o.b)

    def __add__(self, o):
        return Color.in_range(self.r + o.r, self.g + o.g, self.b + o.b)


BLACK = Color(0.0, 0.0, 0.0, 1.0)


def to_u8(c):
    v = c * 255.0
    if not v > 0.0:
        return 0
    if v >= 255.0:
        return 255
    return int(v)


# ----------------------------------------------------------------------------- transformation.rs
def transform_vector(v, m):
    return Vector(m[0][0] * v.x + m[0][1] * v.y + m[0][2] * v.z + m[0][3],
                  m[1][0] * v.x + m[1][1] * v.y + m[1][2] * v.z + m[1][3],
                  m[2][0] * v.x + m[2][1] * v.y + m[2][2] * v.z + m[2][3])


def multiply(m1, m2):
    res = [[0.0] * 4 for _ in range(4)]
    for i in range(4):
        for j in range(4):
            for k in range(4):
                res[i][j] += m1[i][k] * m2[k][j]
    return res


def identity():
    return [[1.0 if i == j else 0.0 for j in range(4)] for i in range(4)]


class MatrixTransformation:
    def __init__(self, m, inv):
        self.m, self.inv = m, inv

    @staticmethod
    def identity():
        return MatrixTransformation(identity(), identity())

    @staticmethod
    def rotation(x, y, z):
        def rx(a):
            c, s = math.cos(a), math.sin(a)
            return [[1.0, 0.0, 0.0, 0.0], [0.0, c, -s, 0.0], [0.0, s, c, 0.0], [0.0, 0.0, 0.0, 1.0]]

        def ry(a):
            c, s = math.cos(a), math.sin(a)
            return [[c, 0.0, -s, 0.0], [0.0, 1.0, 0.0, 0.0], [s, 0.0, c, 0.0], [0.0, 0.0, 0.0, 1.0]]

        def rz(a):
            c, s = math.cos(a), math.sin(a)
            return [[c, -s, 0.0, 0.0], [s, c, 0.0, 0.0], [0.0, 0.0, 1.0, 0.0], [0.0, 0.0, 0.0, 1.0]]
        m = multiply(multiply(rx(x), ry(y)), rz(z))
        inv = multiply(multiply(rx(-x), ry(-y)), rz(-z))
        return MatrixTransformation(m, inv)

    @staticmethod
    def translation(x, y, z):
        m, inv = identity(), identity()
        m[0][3], m[1][3], m[2][3] = x, y, z
        inv[0][3], inv[1][3], inv[2][3] = -x, -y, -z
        return MatrixTransformation(m, inv)

    @staticmethod
    def scaling(x, y, z):
        m, inv = identity(), identity()
        m[0][0], m[1][1], m[2][2] = x, y, z
        inv[0][0], inv[1][1], inv[2][2] = 1.0 / x, 1.0 / y, 1.0 / z
        return MatrixTransformation(m, inv)

    def compose_with(self, other):
        return MatrixTransformation(multiply(other.m, self.m), multiply(self.inv, other.inv))

    def transform_vector(self, v):
        return transform_vector(v, self.m)

    def reverse_transform_vector(self, v):
        return transform_vector(v, self.inv)

    def transform_direction_vector(self, v):
        return transform_vector(v, self.m) - transform_vector(Vector(0.0, 0.0, 0.0), self.m)

    def reverse_transform_direction_vector(self, v):
        return transform_vector(v, self.inv) - transform_vector(Vector(0.0, 0.0, 0.0), self.inv)

    def reverse_transform_ray(self, ray):
        return (self.reverse_transform_vector(ray[0]), self.reverse_transform_direction_vector(ray[1]))


# ----------------------------------------------------------------------------- math_shapes.rs
class Sphere:
    def __init__(self, t, center, radius):
        self.t, self.center, self.radius = t, center, radius

    def reverse_transform_ray(self, ray):
        return self.t.reverse_transform_ray(ray)

    def intersects(self, ray, add):
        point, direction = ray
        v = point - self.center
        d = direction.normalized()
        scale = div(1.0, direction.length())
        r = self.radius
        vd = v.dot(d)
        s = vd * vd - (v.dot(v) - r * r)
        if s < 0.0:
            return
        add((-vd + math.sqrt(s)) * scale)
        add((-vd - math.sqrt(s)) * scale)

    def get_normal(self, p):
        p = self.t.reverse_transform_vector(p)
        return self.t.transform_direction_vector(p - self.center).normalized()

    def is_inside(self, p):
        p = self.t.reverse_transform_vector(p)
        return (p - self.center).length() <= self.radius + EPSILON

    def is_on_surface(self, p):
        p = self.t.reverse_transform_vector(p)
        return abs((p - self.center).length() - self.radius) < EPSILON

    def get_uv(self, p):
        p = self.t.reverse_transform_vector(p - self.center)
        p = p.normalized().scale(1.0 - EPSILON)
        up, u_zero, u_qrtr = Vector(0.0, 1.0, 0.0), Vector(0.0, 0.0, -1.0), Vector(-1.0, 0.0, 0.0)
        phi = acos(-(up.dot(p)))
        if phi != phi:
            phi = 0.0
        th = acos(div(p.dot(u_zero), sin(phi))) / (2.0 * PI)
        if th != th:
            th = 0.0
        v = phi / PI
        u = 1.0 - th if u_qrtr.dot(p) > 0.0 else th
        return (u, v)


class Plane:
    def __init__(self, t, a, b, c, d):
        self.t, self.a, self.b, self.c, self.d = t, a, b, c, d
        self.normal = t.transform_direction_vector(Vector(a, b, c).normalized()).normalized()

    def reverse_transform_ray(self, ray):
        return self.t.reverse_transform_ray(ray)

    def on_plane(self, p):
        return abs(self.a * p.x + self.b * p.y + self.c * p.z + self.d) < EPSILON

    def intersects(self, ray, add):
        p_n = Vector(self.a, self.b, self.c).normalized()
        v_d = p_n.dot(ray[1])
        if v_d != 0.0:
            t = -(p_n.dot(ray[0]) + self.d) * (1.0 / v_d)
            if t >= 0.0:
                add(t)

    def get_normal(self, p):
        return self.normal

    def is_inside(self, p):
        return False

    def is_on_surface(self, p):
        return self.on_plane(self.t.reverse_transform_vector(p))

    def get_uv(self, p):
        return None


class Cube:
    def __init__(self, t, center, length):
        length = length / 2.0
        self.t, self.center, self.length = t, center, length
        c = center
        self.p1 = Plane(t, 0.0, 0.0, 1.0, -(c.z + length / 2.0))
        self.p6 = Plane(t, 0.0, 0.0, -1.0, c.z + -length / 2.0)
        self.p2 = Plane(t, 0.0, 1.0, 0.0, -(c.y + length / 2.0))
        self.p5 = Plane(t, 0.0, -1.0, 0.0, c.y + -length / 2.0)
        self.p3 = Plane(t, 1.0, 0.0, 0.0, -(c.x + length / 2.0))
        self.p4 = Plane(t, -1.0, 0.0, 0.0, c.x + -length / 2.0)

    def reverse_transform_ray(self, ray):
        return self.t.reverse_transform_ray(ray)

    def intersects(self, ray, add):
        t_near, t_far = -INF, INF
        dv = (ray[1].x, ray[1].y, ray[1].z)
        pv = (ray[0].x, ray[0].y, ray[0].z)
        cv = (self.center.x, self.center.y, self.center.z)
        for i in range(3):
            if dv[i] == 0.0:
                if pv[i] < cv[i] - self.length or pv[i] > cv[i] + self.length:
                    return
                continue
            t1 = (cv[i] - self.length - pv[i]) / dv[i]
            t2 = (cv[i] + self.length - pv[i]) / dv[i]
            if t1 > t2:
                t1, t2 = t2, t1
            if t1 > t_near:
                t_near = t1
            if t2 < t_far:
                t_far = t2
            if t_near > t_far or t_far < 0.0:
                return
        add(t_near)
        add(t_far)

    def get_normal(self, p):
        p = self.t.reverse_transform_vector(p)
        for pl in (self.p1, self.p2, self.p3, self.p4, self.p5, self.p6):
            if pl.on_plane(p):
                return pl.normal
        return Vector(1.0, 1.0, 1.0)

    def is_inside(self, p):
        p = self.t.reverse_transform_vector(p)
        c, l = self.center, self.length
        return (p.x <= c.x + l and p.x >= c.x - l and p.y <= c.y + l and p.y >= c.y - l and
                p.z <= c.z + l and p.z >= c.z - l)

    def is_on_surface(self, p):
        p = self.t.reverse_transform_vector(p)
        c, l = self.center, self.length

        def between(x, s, e):
            return s <= x <= e
        if (between(p.y, c.y - l - EPSILON, c.y + l + EPSILON) and between(p.x, c.x - l - EPSILON, c.x + l + EPSILON)
                and (self.p1.on_plane(p) or self.p6.on_plane(p))):
            return True
        if (between(p.z, c.z - l - EPSILON, c.z + l + EPSILON) and between(p.x, c.x - l - EPSILON, c.x + l + EPSILON)
                and (self.p2.on_plane(p) or self.p5.on_plane(p))):
            return True
        if (between(p.y, c.y - l - EPSILON, c.y + l + EPSILON) and between(p.z, c.z - l - EPSILON, c.z + l + EPSILON)
                and (self.p3.on_plane(p) or self.p4.on_plane(p))):
            return True
        return False

    def get_uv(self, p):
        return None


# ----------------------------------------------------------------------------- csg.rs / rt_object.rs
class RTObject:
    def __init__(self, shape, material):
        self.shape, self.material = shape, material

    def intersects(self, ray, add):
        self.shape.intersects(self.shape.reverse_transform_ray(ray), add)


class CSG:
    def __init__(self, a_obj, b_obj, op):
        self.a_obj, self.b_obj, self.op = a_obj, b_obj, op

    def reverse_transform_ray(self, ray):
        return ray

    def intersects(self, ray, add):
        a, b = self.a_obj.shape, self.b_obj.shape
        point, direction = ray

        def keep(other, want):
            def f(d):
                inside = other.is_inside(point + direction.scale(d))
                if inside == want:
                    add(d)
            return f
        if self.op == "union":
            fa, fb = keep(b, False), keep(a, False)
        elif self.op == "intersection":
            fa, fb = keep(b, True), keep(a, True)
        else:
            fa, fb = keep(b, False), keep(a, True)
        self.a_obj.intersects(ray, fa)
        self.b_obj.intersects(ray, fb)

    def get_normal(self, p):
        a, b = self.a_obj.shape, self.b_obj.shape
        if a.is_on_surface(p):
            return a.get_normal(p)
        if b.is_on_surface(p):
            n = b.get_normal(p)
            return n.scale(-1.0) if self.op == "difference" else n
        return Vector(1.0, 0.0, 0.0)

    def is_inside(self, p):
        a, b = self.a_obj.shape, self.b_obj.shape
        if self.op == "union":
            return a.is_inside(p) or b.is_inside(p)
        if self.op == "intersection":
            return a.is_inside(p) and b.is_inside(p)
        return a.is_inside(p) and not b.is_inside(p)

    def is_on_surface(self, p):
        a, b = self.a_obj.shape, self.b_obj.shape
        if self.op == "union":
            return (a.is_on_surface(p) and not b.is_inside(p)) or (b.is_on_surface(p) and not a.is_inside(p))
        if self.op == "intersection":
            return (a.is_on_surface(p) and b.is_inside(p)) or (b.is_on_surface(p) and a.is_inside(p))
        return (a.is_on_surface(p) and not b.is_inside(p)) or (b.is_on_surface(p) and a.is_inside(p))

    def get_uv(self, p):
        a, b = self.a_obj.shape, self.b_obj.shape
        if a.is_on_surface(p):
            return a.get_uv(p)
        if b.is_on_surface(p):
            return b.get_uv(p)
        return None


# ----------------------------------------------------------------------------- material.rs / texture.rs
class Material:
    def __init__(self, color=None, texture=None, reflectivity=0.0, transparency=0.0):
        self.color, self.texture = color, texture
        self.reflectivity, self.transparency = reflectivity, transparency

    def color_at(self, uv):
        if self.texture is None:
            return self.color
        w, h, pix = self.texture
        x = uv[0] * float(w - 1)
        y = float(h) - (uv[1] * float(h - 1)) - 1.0
        xi = 0 if not x > 0.0 else min(int(x), w - 1)
        yi = 0 if not y > 0.0 else min(int(y), h - 1)
        return pix[yi * w + xi]


# ----------------------------------------------------------------------------- camera.rs / raytracer.rs
class Camera:
    def __init__(self, w, h, center):
        self.w, self.h, self.center = w, h, center
        self.up = Vector(0.0, 1.0, 0.0)
        self.direction = (Vector(0.0, 0.0, 0.0) - center).normalized()
        self.aspect = float(w) / float(h)
        right = Vector(0.0, 0.0, 0.0)
        self.right = -Vector.cross(self.direction, self.up) if right.length() == 0.0 else right

    def create_ray(self, x, y):
        sx = ((x / float(self.w)) - 0.5) * self.aspect
        sy = (float(self.h) - 1.0 - y) / float(self.h) - 0.5
        return (self.center, self.direction + self.right.scale(sx) + self.up.scale(sy))


class RayTracer:
    def __init__(self, w, h):
        self.w, self.h = w, h
        self.camera = Camera(w, h, Vector(0.0, 0.0, -100.0))
        self.max_depth = 10
        self.objects, self.lights = [], []
        self.stack = [MatrixTransformation.identity()]

    def add_test_objects(self):
        self.lights.append((Vector(-10.0, 30.0, -50.0), Color.in_range(0.5, 0.5, 0.5)))

    def get_ray_color(self, ray, depth):
        best = [INF, None]
        for obj in self.objects:
            def add(d, obj=obj):
                if d > EPSILON and d < best[0]:
                    best[0], best[1] = d, obj
            obj.intersects(ray, add)
        if best[1] is None:
            return BLACK
        dist, obj = best
        point = ray[0] + ray[1].scale(dist)
        normal = obj.shape.get_normal(point).normalized()
        uv = obj.shape.get_uv(point) or (0.0, 0.0)
        c = obj.material.color_at(uv)
        final = c * Color.in_range(1.0, 1.0, 1.0).intensify(0.6)
        for lp, lcol in self.lights:
            sdir = (lp - point).normalized()
            dl = (lp - point).length()
            tr = [1.0]
            for o in self.objects:
                def add_s(d, o=o):
                    if d > EPSILON and d < dl:
                        tr[0] *= o.material.transparency
                o.intersects((point, sdir), add_s)
            if tr[0] == 0.0:
                continue
            ang = Vector.angle(sdir, normal)
            if ang >= PI / 2.0:
                ang = PI - ang
            inten = 1.0 - (ang / (PI / 2.0)) if (ang < PI / 2.0 and ang >= 0.0) else 0.0
            final = final + c * lcol.intensify(inten).intensify(tr[0])
        ang = Vector.angle(ray[1].scale(-1.0), normal)
        if ang >= PI / 2.0:
            r1, r2, normal, inside = 1.45, 1.0, normal.scale(-1.0), True
        else:
            r1, r2, inside = 1.0, 1.45, False
        t, refl = obj.material.transparency, obj.material.reflectivity
        tir = False
        if depth < self.max_depth and t != 0.0:
            i, r = ray[1], r1 / r2
            cos1 = i.scale(-1.0).dot(normal)
            v = 1.0 - r * r * (1.0 - cos1 * cos1)
            tir = v < 0.0
            if not tir:
                dirn = (i.scale(r) + normal.scale(r * cos1 - math.sqrt(v))).normalized()
                rc = self.get_ray_color((point, dirn), depth + 1)
                final = final.intensify(1.0 - t) + rc.intensify(t)
        if tir:
            refl = refl + (1.0 - refl) * t
        if depth < self.max_depth and refl != 0.0 and (not inside or tir):
            i = ray[1]
            dirn = i - normal.scale(2.0).scale(normal.dot(i))
            rc = self.get_ray_color((point, dirn), depth + 1)
            final = final.intensify(1.0 - refl) + rc.intensify(refl)
        return final

    def get_pixel(self, x, y):
        return self.get_ray_color(self.camera.create_ray(float(x), float(y)), 0)


# ----------------------------------------------------------------------------- scene DSL
class DSLError(Exception):
    pass


class ParseError(DSLError):
    pass


_WS = re.compile(r"(?:[ \n\r]|//[^\n]*(?:\n|$))*")
_IDENT = re.compile(r"[A-Za-z_][A-Za-z0-9_]*")
_NUMBER = re.compile(r"[0-9]+(?:\.[0-9]+)?")
_KEYWORDS = ("local", "scale", "rotate", "translate", "draw", "display", "append",
             "sphere", "plane", "csg", "cube", "function")
_COLORS = {"red": (1.0, 0.0, 0.0), "orange": (1.0, 0.5, 0.0), "yellow": (1.0, 1.0, 0.0),
           "green": (0.0, 1.0, 0.0), "blue": (0.0, 0.0, 1.0), "purple": (1.0, 0.0, 1.0),
           "black": (0.0, 0.0, 0.0), "white": (1.0, 1.0, 1.0)}


class _P:
    """Backtracking PEG parser for scene_grammar.pest producing tuples."""

    def __init__(self, s):
        self.s, self.i = s, 0

    def ws(self):
        self.i = _WS.match(self.s, self.i).end()

    def lit(self, t):
        if self.s.startswith(t, self.i):
            self.i += len(t)
            return True
        return False

    def kw(self, *words):
        for w in words:
            if self.s.startswith(w, self.i):
                j = self.i + len(w)
                if j < len(self.s) and (self.s[j].isalnum() and self.s[j].isascii() or self.s[j] == "_"):
                    continue
                self.i = j
                return w
        return None

    def ident(self):
        save = self.i
        if self.kw(*_KEYWORDS):
            self.i = save
            return None
        m = _IDENT.match(self.s, self.i)
        if not m:
            return None
        self.i = m.end()
        return m.group()

    def one_ws(self):
        m = re.compile(r"[ \n\r]|//[^\n]*(?:\n|$)").match(self.s, self.i)
        if m:
            self.i = m.end()
            return True
        return False

    def try_(self, f):
        save = self.i
        r = f()
        if r is None:
            self.i = save
        return r

    def params(self):
        out = []
        while True:
            save = self.i
            if out:
                self.ws()
            e = self.try_(self.expr)
            if e is None:
                self.i = save
                return out
            out.append(e)
            s2 = self.i
            self.ws()
            if not self.lit(","):
                self.i = s2

    def value(self):
        m = _NUMBER.match(self.s, self.i)
        if m and not (m.end() < len(self.s) and self.s[m.end()].isascii() and self.s[m.end()].isalpha()):
            self.i = m.end()
            return ("num", float(m.group()))
        for f in (self._color_name, self._rgb, self._vector, self._texture, self._paren, self._object,
                  self._string, self._ref):
            r = self.try_(f)
            if r is not None:
                return r
        return None

    def _color_name(self):
        w = self.kw(*_COLORS)
        return ("color", _COLORS[w] + (1.0,)) if w else None

    def _rgb(self):
        if not self.lit("rgb"):
            return None
        self.ws()
        if not self.lit("("):
            return None
        parts = []
        for _ in range(3):
            self.ws()
            e = self.expr()
            if e is None:
                return None
            parts.append(e)
            s2 = self.i
            self.ws()
            if not self.lit(","):
                self.i = s2
        self.ws()
        return ("rgb", parts) if self.lit(")") else None

    def _vector(self):
        if not self.lit("<"):
            return None
        parts = []
        for k in range(3):
            self.ws()
            e = self.expr()
            if e is None:
                return None
            parts.append(e)
            self.ws()
            if not self.lit("," if k < 2 else ">"):
                return None
        return ("vec", parts)

    def _texture(self):
        if not self.lit("texture"):
            return None
        self.ws()
        if not self.lit("("):
            return None
        self.ws()
        e = self.expr()
        if e is None:
            return None
        self.ws()
        return ("tex", e) if self.lit(")") else None

    def _paren(self):
        if not self.lit("("):
            return None
        self.ws()
        e = self.expr()
        if e is None:
            return None
        self.ws()
        return e if self.lit(")") else None

    def _object(self):
        name = self.kw("sphere", "plane", "csg", "cube")
        if not name:
            return None
        self.ws()
        if not self.lit("("):
            return None
        self.ws()
        ps = self.params()
        self.ws()
        return ("obj", name, ps) if self.lit(")") else None

    def _string(self):
        m = re.compile(r"\"([^\"]*)\"|'([^']*)'").match(self.s, self.i)
        if not m:
            return None
        self.i = m.end()
        return ("str", m.group(1) if m.group(1) is not None else m.group(2))

    def _ref(self):
        n = self.ident()
        return ("ref", n) if n else None

    def neg(self):
        save = self.i
        minus = self.lit("-")
        if minus:
            self.ws()
        v = self.value()
        if v is None:
            self.i = save
            return None
        return ("neg", v) if minus else v

    def chain(self, sub, ops):
        left = sub()
        if left is None:
            return None
        result = None
        while True:
            save = self.i
            self.ws()
            if self.i < len(self.s) and self.s[self.i] in ops:
                op = self.s[self.i]
                self.i += 1
                self.ws()
                right = sub()
                if right is None:
                    self.i = save
                    break
                if result is None:            # later operators of the chain are dropped
                    result = ("bin", op, left, right)
            else:
                self.i = save
                break
        return result if result is not None else left

    def mult(self):
        return self.chain(self.neg, "*/%")

    def expr(self):
        return self.chain(self.mult, "+-")

    def bool_expr(self):
        a = self.expr()
        if a is None:
            return None
        self.ws()
        if self.i < len(self.s) and self.s[self.i] in "<>":
            op = self.s[self.i]
            self.i += 1
            self.ws()
            b = self.expr()
            if b is not None:
                return ("bin", op, a, b)
        return None

    def statement(self):
        for f in (self._camera, self._light, self._do, self._if, self._while, self._call, self._function,
                  self._command, self._assign, self._xform):
            r = self.try_(f)
            if r is not None:
                return r
        return None

    def _camera(self):
        if not (self.lit("set") and self.one_ws() and self.kw("camera")):
            return None
        self.ws()
        if not self.lit("("):
            return None
        self.ws()
        e = self.expr()
        if e is None:
            return None
        self.ws()
        return ("camera", e) if self.lit(")") else None

    def _light(self):
        if not (self.lit("append") and self.one_ws() and self.kw("light")):
            return None
        self.ws()
        if not self.lit("("):
            return None
        self.ws()
        ps = self.params()
        self.ws()
        return ("light", ps) if self.lit(")") else None

    def _do(self):
        if not self.kw("do"):
            return None
        self.ws()
        body = self.stmts()
        self.ws()
        return body if self.kw("end") else None

    def _cond(self, key, sep, kind):
        if not self.kw(key):
            return None
        self.ws()
        c = self.bool_expr()
        if c is None:
            return None
        self.ws()
        if not self.kw(sep):
            return None
        self.ws()
        body = self.stmts()
        self.ws()
        return (kind, c, body) if self.kw("end") else None

    def _if(self):
        return self._cond("if", "then", "if")

    def _while(self):
        return self._cond("while", "do", "while")

    def _call(self):
        if not self.kw("call"):
            return None
        self.ws()
        n = self.ident()
        if not n:
            return None
        self.ws()
        if not self.lit("("):
            return None
        self.ws()
        ps = self.params()
        self.ws()
        return ("call", n, ps) if self.lit(")") else None

    def _function(self):
        if not self.kw("function"):
            return None
        self.ws()
        n = self.ident()
        if not n:
            return None
        self.ws()
        if not self.lit("("):
            return None
        names = []
        while True:
            save = self.i
            self.ws()
            p = self.ident()
            if not p:
                self.i = save
                break
            names.append(p)
            s2 = self.i
            self.ws()
            if not self.lit(","):
                self.i = s2
        self.ws()
        if not self.lit(")"):
            return None
        self.ws()
        body = self.stmts()
        self.ws()
        return ("function", n, names, body) if self.kw("end") else None

    def _command(self):
        c = self.kw("draw", "display", "append")
        if not c:
            return None
        self.ws()
        if not self.lit("("):
            return None
        self.ws()
        ps = self.params()
        self.ws()
        return ("command", c, ps) if self.lit(")") else None

    def _assign(self):
        local = bool(self.kw("local"))
        if local:
            self.ws()
        n = self.ident()
        if not n:
            return None
        self.ws()
        if not self.lit("="):
            return None
        self.ws()
        e = self.expr()
        return ("assign", local, n, e) if e is not None else None

    def _xform(self):
        k = self.kw("scale", "rotate", "translate")
        if not k:
            return None
        self.ws()
        if not self.lit("("):
            return None
        parts = []
        for j in range(3):
            self.ws()
            e = self.expr()
            if e is None:
                return None
            parts.append(e)
            self.ws()
            if not self.lit("," if j < 2 else ")"):
                return None
        self.ws()
        body = self.statement()
        return ("xform", k, parts, body) if body is not None else None

    def stmts(self):
        out = []
        while True:
            save = self.i
            if out:
                self.ws()
            st = self.try_(self.statement)
            if st is None:
                self.i = save
                return ("block", out)
            out.append(st)


def _walk_commands(node, acc):
    if isinstance(node, tuple):
        if node and node[0] == "command":
            acc.append(node[1])
        for x in node:
            _walk_commands(x, acc)
    elif isinstance(node, list):
        for x in node:
            _walk_commands(x, acc)


class Scene:
    """load_scene(RayTracer::new_default + add_test_objects, time) -- scene_loader.rs:24-47."""

    def __init__(self, text, time, w, h, textures, max_depth=10):
        self.rt = RayTracer(w, h)
        self.rt.add_test_objects()
        self.rt.max_depth = max_depth
        self.textures = textures
        p = _P(text)
        p.ws()
        ast = p.stmts()
        p.ws()
        if p.i != len(text):
            raise ParseError(f"parse error near offset {p.i}")
        cmds = []
        _walk_commands(ast, cmds)
        if any(c != "draw" for c in cmds):
            raise DSLError("not implemented")
        self.globals = {"time": ("num", time)}
        self.frames = []
        self.functions = {}
        self.exec(ast)

    # -- evaluation (ast_node.rs:150-265, 438-596)
    def locals(self):
        return self.frames[-1] if self.frames else self.globals

    def num(self, v):
        if v[0] != "num":
            raise DSLError("Cannot convert value to number")
        return v[1]

    def ev(self, e):
        k = e[0]
        if k in ("num", "color", "str"):
            return e
        if k == "ref":
            if e[1] in self.locals():
                return self.locals()[e[1]]
            if e[1] in self.globals:
                return self.globals[e[1]]
            raise DSLError("unknown variable " + e[1])
        if k == "vec":
            return ("vecv", tuple(self.num(self.ev(x)) for x in e[1]))
        if k == "rgb":
            return ("color", tuple(self.num(self.ev(x)) for x in e[1]) + (1.0,))
        if k == "tex":
            f = self.ev(e[1])
            if f[0] != "str":
                raise DSLError("Cannot convert value to string")
            return ("texv", self.textures[f[1]])
        if k == "neg":
            v = self.ev(e[1])
            if v[0] == "num":
                return ("num", -v[1])
            if v[0] == "vecv":
                return ("vecv", tuple(-c for c in v[1]))
            raise DSLError("Cannot apply -")
        if k == "obj":
            return self.obj(e[1], [self.ev(x) for x in e[2]])
        if k == "bin":
            op, a, b = e[1], self.ev(e[2]), self.ev(e[3])
            if op == "+":
                return ("num", self.num(a) + self.num(b))
            if op == "-":
                return ("num", self.num(a) - self.num(b))
            if op in "*/":
                f = (lambda x, y: x * y) if op == "*" else (lambda x, y: x / y)
                if a[0] == "num" and b[0] == "num":
                    return ("num", f(a[1], b[1]))
                for x, n in ((a, b), (b, a)):
                    if n[0] == "num" and x[0] in ("color", "vecv"):
                        return (x[0], tuple(f(c, n[1]) for c in x[1]))
                raise DSLError("bad operands")
            if op in "<>":
                if a[0] != "num" or b[0] != "num":
                    raise DSLError("Cannot compare")
                return ("bool", a[1] < b[1] if op == "<" else a[1] > b[1])
            raise DSLError("Operator Modulo not yet implemented")
        raise DSLError("bad expression")

    def obj(self, name, vals):
        by = {"num": [], "str": [], "vecv": [], "objv": [], "color": [], "texv": []}
        for v in vals:
            if v[0] not in by:
                raise DSLError("Unexpected argument type")
            by[v[0]].append(v[1])

        def pop(kind, default):
            return by[kind].pop(0) if by[kind] else default
        shape = {"kind": name, "t": self.rt.stack[-1]}
        if name in ("sphere", "cube"):
            shape["center"] = pop("vecv", (0.0, 0.0, 0.0))
            shape["size"] = pop("num", 1.0)
        elif name == "plane":
            shape["normal"] = pop("vecv", (0.0, 1.0, 0.0))
            shape["distance"] = pop("num", 1.0)
        else:
            op = pop("str", "union")
            if op not in ("union", "intersection", "difference"):
                raise DSLError("Unknown CSG operator")
            if len(by["objv"]) < 2:
                raise DSLError("Expected object")
            shape["op"], shape["a"], shape["b"] = op, by["objv"].pop(0), by["objv"].pop(0)
        tex = pop("texv", None)
        shape["texture"] = tex
        shape["color"] = None if tex is not None else pop("color", (0.0, 0.0, 0.0, 1.0))
        shape["reflectivity"] = pop("num", 0.0)
        shape["transparency"] = pop("num", 0.0)
        if any(by.values()):
            raise DSLError("assertion failed: unused arguments")
        return ("objv", shape)

    def to_rt_object(self, sh):                               # sceneparser/shape.rs:42-93
        mat = Material(None if sh["texture"] is not None else Color(*sh["color"]), sh["texture"],
                       sh["reflectivity"], sh["transparency"])
        k = sh["kind"]
        if k == "sphere":
            shape = Sphere(sh["t"], Vector(*sh["center"]), sh["size"])
        elif k == "cube":
            shape = Cube(sh["t"], Vector(*sh["center"]), sh["size"])
        elif k == "plane":
            n = sh["normal"]
            shape = Plane(sh["t"], n[0], n[1], n[2], sh["distance"])
        else:
            shape = CSG(self.to_rt_object(sh["a"]), self.to_rt_object(sh["b"]), sh["op"])
        return RTObject(shape, mat)

    def exec(self, st):
        k = st[0]
        if k == "block":
            for s in st[1]:
                self.exec(s)
        elif k == "assign":
            v = self.ev(st[3])
            (self.locals() if st[1] else self.globals)[st[2]] = v
        elif k == "function":
            self.functions[st[1]] = st
        elif k == "call":
            vals = [self.ev(x) for x in st[2]]
            f = self.functions.get(st[1])
            if f is None or len(f[2]) != len(vals):
                raise DSLError("bad call")
            self.frames.append(dict(zip(f[2], vals)))
            self.exec(f[3])
            self.frames.pop()
        elif k == "command":
            vals = [self.ev(x) for x in st[2]]
            if len(vals) != 1 or vals[0][0] != "objv":
                raise DSLError("draw needs one object")
            self.rt.objects.append(self.to_rt_object(vals[0][1]))
        elif k == "xform":
            x, y, z = (self.num(self.ev(e)) for e in st[2])
            t = {"translate": MatrixTransformation.translation, "rotate": MatrixTransformation.rotation,
                 "scale": MatrixTransformation.scaling}[st[1]](x, y, z)
            self.rt.stack.append(t.compose_with(self.rt.stack[-1]))
            self.exec(st[3])
            self.rt.stack.pop()
        elif k in ("if", "while"):
            while True:
                c = self.ev(st[1])
                if c[0] != "bool":
                    raise DSLError("Cannot convert value to boolean")
                if not c[1]:
                    break
                self.exec(st[2])
                if k == "if":
                    break
        elif k == "light":
            vals = [self.ev(x) for x in st[1]]
            col = next((v[1] for v in vals if v[0] == "color"), (0.5, 0.5, 0.5, 1.0))
            pt = next((v[1] for v in vals if v[0] == "vecv"), (0.0, 0.0, 0.0))
            self.rt.lights.append((self.rt.stack[-1].transform_vector(Vector(*pt)), Color(*col)))
        elif k == "camera":
            v = self.ev(st[1])
            if v[0] != "vecv":
                raise DSLError("Cannot convert value to vector")
            c = self.rt.stack[-1].transform_vector(Vector(*v[1]))
            c = self.rt.stack[-1].transform_vector(c)
            self.rt.camera = Camera(self.rt.w, self.rt.h, c)

    def render(self, rows=None):
        """[(r, g, b, a) f64 for each pixel] row-major for the given rows (default all)."""
        rows = range(self.rt.h) if rows is None else rows
        return [[self.rt.get_pixel(x, y) for x in range(self.rt.w)] for y in rows]


def load_texture(rgba8) -> tuple:
    """(w, h, [Color]) from an (h, w, 4) uint8 array, /255.0 as sceneparser/texture.rs:29-33."""
    h, w = rgba8.shape[:2]
    flat = rgba8.reshape(-1, 4).tolist()
    return (w, h, [Color(p[0] / 255.0, p[1] / 255.0, p[2] / 255.0, p[3] / 255.0) for p in flat])


def antialias(scene, frame_u8, threshold=0.01, level=3):
    """antialiaser.rs:87-191 over a quantised frame (list of rows of (r, g, b, a) u8 tuples),
    as debug_window.rs:275-320 drives it.  Returns (rows of Color, rays traced); the last row and
    column are the source colours."""
    H, W = len(frame_u8), len(frame_u8[0])
    size = (1 << level) + 1

    def src(x, y):                                                  # easy_pixbuf.rs:55-64
        p = frame_u8[y][x]
        return Color(p[0] / 255.0, p[1] / 255.0, p[2] / 255.0, p[3] / 255.0)

    def different(c1, c2):                                          # antialiaser.rs:154-162
        return (abs(c1.r - c2.r) + abs(c1.g - c2.g) + abs(c1.b - c2.b) + abs(c1.a - c2.a)) / 4.0 > threshold

    def average(c1, c2, c3, c4):                                    # antialiaser.rs:164-171
        return Color((c1.r + c2.r + c3.r + c4.r) / 4.0, (c1.g + c2.g + c3.g + c4.g) / 4.0,
                     (c1.b + c2.b + c3.b + c4.b) / 4.0, (c1.a + c2.a + c3.a + c4.a) / 4.0)

    rays = 0
    out = []
    for y in range(H - 1):
        row = []
        for x in range(W - 1):
            n = size - 1
            memo = {(0, 0): src(x, y), (0, n): src(x, y + 1), (n, 0): src(x + 1, y), (n, n): src(x + 1, y + 1)}

            def sub(sx, sy):
                nonlocal rays
                if (sx, sy) not in memo:
                    rays += 1
                    memo[(sx, sy)] = scene.rt.get_pixel(x + (sx / size), y + (sy / size))
                return memo[(sx, sy)]

            def cell(x1, y1, x2, y2, lv):
                c1, c2, c3, c4 = sub(x1, y1), sub(x2, y1), sub(x1, y2), sub(x2, y2)
                if not (different(c1, c2) or different(c1, c3) or different(c1, c4)) or lv <= 0:
                    return average(c1, c2, c3, c4)
                mx, my = x1 + (x2 - x1) // 2, y1 + (y2 - y1) // 2
                return average(cell(x1, y1, mx, my, lv - 1), cell(mx, y1, x2, my, lv - 1),
                               cell(x1, my, mx, y2, lv - 1), cell(mx, my, x2, y2, lv - 1))

            row.append(cell(0, 0, n, n, level))
        row.append(src(W - 1, y))
        out.append(row)
    out.append([src(x, H - 1) for x in range(W)])
    return out, rays
