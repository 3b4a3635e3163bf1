"""Triangle primitive (reference `geometry/triangle.py:8-86`).

The reference `Triangle.__init__` passes `assigned_primitive=` to a collider whose constructor
takes `assigned_surface` (triangle.py:12 vs :20) and so raises TypeError; the collider works when
built directly.  Here both spellings are accepted so the primitive is usable; the collider's
intersection is the reference's (plane through the centroid + three edge half-spaces).
`get_uv` is undefined in the reference (uses unset pu/pv/w/h), so textured triangles are rejected
at scene lowering.
"""
from .primitive import Primitive
from .collider import Collider

__all__ = ["Triangle", "Triangle_Collider"]


class Triangle(Primitive):
    def __init__(self, center, material, p1, p2, p3, max_ray_depth=5, shadow=True):
        super().__init__(center, material, max_ray_depth, shadow=shadow)
        self.collider_list += [Triangle_Collider(assigned_primitive=self, p1=p1, p2=p2, p3=p3)]


class Triangle_Collider(Collider):
    """Device: `rt_triangle_hit`."""

    def __init__(self, assigned_surface=None, p1=None, p2=None, p3=None, assigned_primitive=None):
        self.assigned_primitive = assigned_primitive if assigned_primitive is not None else assigned_surface
        self.p1 = p1
        self.p2 = p2
        self.p3 = p3
        self.normal = ((self.p2 - self.p1).cross(self.p3 - self.p1)).normalize()
        self.centroid = (self.p1 + self.p2 + self.p3) / 3
        self.center = self.centroid
        self.n31 = (self.p3 - self.p1).cross(self.normal)
        self.n12 = (self.p1 - self.p2).cross(self.normal)
        self.n23 = (self.p2 - self.p3).cross(self.normal)

    def rotate(self, M, center):
        self.p1 = center + (self.p1 - center).matmul(M)
        self.p2 = center + (self.p2 - center).matmul(M)
        self.p3 = center + (self.p3 - center).matmul(M)
        self.n31 = self.n31.matmul(M)
        self.n12 = self.n12.matmul(M)
        self.n23 = self.n23.matmul(M)
        self.normal = self.normal.matmul(M)
        self.centroid = center + (self.centroid - center).matmul(M)

    def get_uv(self, hit):
        # triangle.py:79-83 reads pu/pv/w/h, which a Triangle_Collider never has
        raise NotImplementedError("Triangle uv is undefined in the reference (triangle.py:79-83)")
