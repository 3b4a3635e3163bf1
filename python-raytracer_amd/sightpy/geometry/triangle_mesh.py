"""OBJ triangle mesh (reference `geometry/triangle_mesh.py:12-43`).

The reference constructor raises NameError (`colliders` undefined, :40), and its header notes the
missing bounding volume hierarchy (:7-9).  This version builds one `Triangle_Collider` per face
(vertex indices from 'f' records, 1-based, '/'-separated), which is what the reference intends.
On the device the Triangle colliders of a scene with 8 or more of them are intersected through a
BVH built when the scene is uploaded (csrc/rt_bvh.h, traversal `bvh_nearest` / `bvh_shadow` in
csrc/rt_device.h), with the same nearest / first-index / tie results as the linear loop over
`scene.collider_list`.
"""
from ..utils.vector3 import vec3
from .primitive import Primitive
from .triangle import Triangle_Collider

__all__ = ["TriangleMesh"]


class TriangleMesh(Primitive):
    def __init__(self, file_name, center, material, max_ray_depth=5, shadow=True):
        super().__init__(center, material, max_ray_depth, shadow=shadow)
        verts, faces = [], []
        with open(file_name, "r") as f:
            for line in f.read().split("\n"):
                tok = line.split()
                if not tok:
                    continue
                if tok[0] == "v":
                    verts.append(vec3(float(tok[1]), float(tok[2]), float(tok[3])))
                elif tok[0] == "f":
                    faces.append([int(t.split("/")[0]) - 1 for t in tok[1:4]])
        for a, b, c in faces:
            self.collider_list += [
                Triangle_Collider(
                    assigned_primitive=self, p1=verts[a] + center, p2=verts[b] + center, p3=verts[c] + center
                )
            ]
