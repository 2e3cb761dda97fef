"""Drop-in mirrors of the reference's ``model/`` classes (SoraKurihara/FFM)."""
from .. import learn_keys as _learn_keys  # noqa: F401  (numpy._core alias for table pickles)
