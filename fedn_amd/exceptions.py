"""Exceptions mirroring fedn/common/exceptions.py:1-10 (same base classes, same names)."""


class ModelError(BaseException):
    pass


class InvalidParameterError(BaseException):
    """Raised by Parameters.validate (fedn/utils/parameters.py:38-51); a BaseException, as in FEDn."""
