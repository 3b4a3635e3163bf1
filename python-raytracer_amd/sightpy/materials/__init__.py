from .material import Material
from .glossy import Glossy
from .refractive import Refractive
from .thin_film_interference import ThinFilmInterference
from .diffuse import Diffuse
from .emissive import Emissive
