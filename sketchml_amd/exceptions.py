"""Exception types mirroring the reference's unchecked exceptions.

base/SketchMLException.java:3-15 and sketch/quantile/QuantileSketchException.java:5-17 are both
RuntimeExceptions; C-ABI status codes map onto them here (and onto the same Java classes in the
JNI shim).
"""
from . import _lib


class SketchMLException(RuntimeError):
    pass


class QuantileSketchException(SketchMLException):
    pass


def check(status: int, what: str = "") -> None:
    """Raise the reference's exception for a non-zero C-ABI status."""
    if status == _lib.SKML_OK:
        return
    msg = _lib.last_error() or f"status {status}"
    if what:
        msg = f"{what}: {msg}"
    if status == _lib.SKML_E_NAN:
        raise QuantileSketchException("Encounter NaN value")
    if status == _lib.SKML_E_ARG and "partition number" in msg:
        raise QuantileSketchException(msg)
    raise SketchMLException(msg)
