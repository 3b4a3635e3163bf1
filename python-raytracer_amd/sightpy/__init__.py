"""sightpy on MI355X: the reference's public API (lmondada/Python-Raytracer `sightpy/__init__.py`)
backed by hand-written HIP kernels for gfx950 (`libsightpy_hip.so`)."""
import numpy as np

from .utils.constants import *
from .utils.vector3 import *
from .utils.colour_functions import *
from .utils.image_functions import *

from .ray import *
from .scene import *
from .geometry import *
from .lights import *
from .materials import *
from .textures.texture import *
from .animation import *

# names the reference leaks through `from sightpy import *` (its modules have no __all__)
import copy, numbers, time
from functools import reduce
from multiprocessing import Pool, cpu_count
from abc import abstractmethod
from pathlib import Path
from PIL import Image, ImageFilter
from .camera import Camera
from .backgrounds.skybox import SkyBox, SkyBox_Material
from .backgrounds.panorama import Panorama
from .utils import colour_functions as cf
from .scene import batch_rays, get_raycolor_tuple
