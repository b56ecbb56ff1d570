"""Score networks (reference: models/__init__.py).  Importing the package
registers 'ncsnpp' and 'ddpm' with `models.utils.register_model`."""
from . import utils, layers, layerspp, up_or_down_sampling  # noqa: F401
from . import ncsnpp, ddpm  # noqa: F401
