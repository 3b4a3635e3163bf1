from .primitive import *
from .collider import *
from .sphere import *
from .plane import *
from .triangle import *
from .triangle_mesh import *
from .cuboid import *
