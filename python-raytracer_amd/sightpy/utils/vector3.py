"""Structure-of-arrays 3-vector used to describe scenes on the host.

API mirror of the reference container (`sightpy/utils/vector3.py:12-234`): three parallel
components that are Python/numpy scalars or numpy arrays.  In this package the container is
*only* a host-side description type (camera placement, primitive centres, colours, IORs and the
ray batches handed to `get_raycolor`); every per-ray computation of the hot path runs in the
HIP kernels under `csrc/`.  Scalar arithmetic here must nonetheless round exactly like the
reference, because the scene constants it produces (plane normals, camera basis, rotated cuboid
bases, Fresnel F0 terms) are uploaded verbatim to the device: every operator below evaluates
the same expression tree, in the same order, as the reference operator it mirrors.
"""
import numbers

import numpy as np

__all__ = ["vec3", "rgb", "extract", "array_to_vec3"]

_AXES = ("x", "y", "z")


def extract(cond, x):
    """`np.extract` that passes scalars through (reference `vector3.py:5-9`)."""
    if isinstance(x, numbers.Number):
        return x
    return np.extract(cond, x)


def _is_operand(v):
    return isinstance(v, (numbers.Number, np.ndarray))


class vec3:
    """Three components; arithmetic is component-wise (reference `vector3.py:12-234`)."""

    __array_priority__ = 1000  # make `ndarray <op> vec3` defer to vec3's reflected operators

    def __init__(self, x, y, z):
        self.x = x
        self.y = y
        self.z = z

    # -- helpers -----------------------------------------------------------------------------
    def _map(self, fn):
        return vec3(fn(self.x), fn(self.y), fn(self.z))

    def _zip(self, other, fn):
        if isinstance(other, vec3):
            return vec3(fn(self.x, other.x), fn(self.y, other.y), fn(self.z, other.z))
        if _is_operand(other):
            return vec3(fn(self.x, other), fn(self.y, other), fn(self.z, other))
        return NotImplemented

    def _rzip(self, other, fn):
        # reflected form: `other <op> self`, operand order preserved
        if isinstance(other, vec3):
            return vec3(fn(other.x, self.x), fn(other.y, self.y), fn(other.z, self.z))
        if _is_operand(other):
            return vec3(fn(other, self.x), fn(other, self.y), fn(other, self.z))
        return NotImplemented

    def __str__(self):
        return "(" + str(self.x) + ", " + str(self.y) + ", " + str(self.z) + ")"

    __repr__ = __str__

    # -- arithmetic (reference vector3.py:31-77) ---------------------------------------------
    def __add__(self, v):
        return self._zip(v, lambda a, b: a + b)

    def __radd__(self, v):
        # reference evaluates `self + v` for the reflected add (vector3.py:37-41)
        return self._zip(v, lambda a, b: a + b)

    def __sub__(self, v):
        return self._zip(v, lambda a, b: a - b)

    def __rsub__(self, v):
        return self._rzip(v, lambda a, b: a - b)

    def __mul__(self, v):
        return self._zip(v, lambda a, b: a * b)

    def __rmul__(self, v):
        return self._rzip(v, lambda a, b: a * b)

    def __truediv__(self, v):
        return self._zip(v, lambda a, b: a / b)

    def __rtruediv__(self, v):
        return self._rzip(v, lambda a, b: a / b)

    def __pow__(self, a):
        return self._map(lambda c: c ** a)

    def __abs__(self):
        return self._map(np.abs)

    def __neg__(self):
        return self * -1.0

    def __eq__(self, other):
        return (self.x == other.x) & (self.y == other.y) & (self.z == other.z)

    __hash__ = None

    def __array_ufunc__(self, ufunc, method, *inputs, **kwargs):
        # numpy >= 2 stopped routing np.abs(vec3) to __abs__; apply unary/binary ufuncs
        # component-wise, which is the behaviour the reference was written against.
        if method != "__call__":
            return NotImplemented
        parts = []
        for ax in _AXES:
            args = [getattr(i, ax) if isinstance(i, vec3) else i for i in inputs]
            parts.append(ufunc(*args, **kwargs))
        return vec3(*parts)

    # -- component utilities -----------------------------------------------------------------
    @staticmethod
    def real(v):
        return vec3(np.real(v.x), np.real(v.y), np.real(v.z))

    @staticmethod
    def imag(v):
        return vec3(np.imag(v.x), np.imag(v.y), np.imag(v.z))

    def yzx(self):
        return vec3(self.y, self.z, self.x)

    def xyz(self):
        return vec3(self.x, self.y, self.z)

    def zxy(self):
        return vec3(self.z, self.x, self.y)

    def average(self):
        return (self.x + self.y + self.z) / 3

    def components(self):
        return (self.x, self.y, self.z)

    def to_array(self):
        return np.array([self.x, self.y, self.z])

    @staticmethod
    def exp(v):
        return vec3(np.exp(v.x), np.exp(v.y), np.exp(v.z))

    @staticmethod
    def sqrt(v):
        return vec3(np.sqrt(v.x), np.sqrt(v.y), np.sqrt(v.z))

    # -- geometry ----------------------------------------------------------------------------
    def dot(self, v):
        return self.x * v.x + self.y * v.y + self.z * v.z

    def square_length(self):
        return self.dot(self)

    def length(self):
        return np.sqrt(self.dot(self))

    def cross(self, v):
        return vec3(
            self.y * v.z - self.z * v.y,
            -self.x * v.z + self.z * v.x,
            self.x * v.y - self.y * v.x,
        )

    def normalize(self):
        mag = self.length()
        return self * (1.0 / np.where(mag == 0, 1, mag))

    def matmul(self, matrix):
        # scalar components -> BLAS gemv, array components -> BLAS gemm (fma chain per row)
        if isinstance(self.x, numbers.Number):
            return array_to_vec3(np.dot(matrix, self.to_array()))
        if isinstance(self.x, np.ndarray):
            return array_to_vec3(np.tensordot(matrix, self.to_array(), axes=([1, 0])))
        raise TypeError("vec3.matmul: unsupported component type %r" % type(self.x))

    def change_basis(self, new_basis):
        return vec3(self.dot(new_basis[0]), self.dot(new_basis[1]), self.dot(new_basis[2]))

    # -- batch utilities ---------------------------------------------------------------------
    def shape(self, *newshape):
        if isinstance(self.x, numbers.Number):
            return 1
        if isinstance(self.x, np.ndarray):
            return self.x.shape
        return None

    def __len__(self):
        shape = self.shape()
        try:
            return shape[0]
        except TypeError:
            return shape

    def __getitem__(self, ind):
        return vec3(self.x[ind], self.y[ind], self.z[ind])

    def broadcast_to(self, shape):
        return self._map(lambda c: np.broadcast_to(c, shape))

    @staticmethod
    def concatenate(vecs):
        return vec3(*(np.concatenate([getattr(v, ax) for v in vecs]) for ax in _AXES))

    def extract(self, cond):
        return self._map(lambda c: extract(cond, c))

    @staticmethod
    def where(cond, out_true, out_false):
        return vec3(*(np.where(cond, getattr(out_true, ax), getattr(out_false, ax)) for ax in _AXES))

    @staticmethod
    def select(mask_list, out_list):
        return vec3(*(np.select(mask_list, [getattr(o, ax) for o in out_list]) for ax in _AXES))

    def clip(self, min, max):
        return self._map(lambda c: np.clip(c, min, max))

    def place(self, cond):
        out = vec3(np.zeros(cond.shape), np.zeros(cond.shape), np.zeros(cond.shape))
        for ax in _AXES:
            np.place(getattr(out, ax), cond, getattr(self, ax))
        return out

    def repeat(self, n):
        return self._map(lambda c: np.repeat(c, n))

    def reshape(self, *newshape):
        return self._map(lambda c: c.reshape(*newshape))

    def mean(self, axis):
        return self._map(lambda c: np.mean(c, axis=axis))


def array_to_vec3(array):
    return vec3(array[0], array[1], array[2])


rgb = vec3
