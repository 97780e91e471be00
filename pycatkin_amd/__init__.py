"""pycatkin_amd -- MI355X-native batched microkinetic (MK) solver with the
PyCatKin System / Reactor API.

All compute runs in the HIP kernels of libpycatkin_amd.so (gfx950); the
Python layer compiles networks and marshals device buffers."""
from .energy import TSYM, Descriptor, LinearForm, clamp0  # noqa: F401
from .classes.state import ScalingState, State  # noqa: F401
from .classes.reaction import Reaction, ReactionDerivedReaction, UserDefinedReaction  # noqa: F401
from .classes.reactor import CSTReactor, InfiniteDilutionReactor, Reactor  # noqa: F401
from .classes.system import SteadyStateResults, System  # noqa: F401
from .classes.solver import SolScore, SteadyStateSolver  # noqa: F401
from .functions.load_input import read_from_input_file  # noqa: F401

__version__ = '0.1.0'
