from .texture import *
