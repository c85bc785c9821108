"""Aggregator hyper-parameters, mirroring fedn/utils/parameters.py:4-51.

``Parameters(dict).validate(schema)`` raises :class:`InvalidParameterError` for a key
outside the schema or a value failing ``isinstance`` (so ``learning_rate=1``, an int,
is rejected exactly like FEDn does).
"""
from .exceptions import InvalidParameterError


class Parameters(dict):
    def __init__(self, parameters=None):
        super().__init__()
        if parameters:
            for key, value in parameters.items():
                self[key] = value

    def validate(self, parameter_schema):
        for key, value in self.items():
            if key not in parameter_schema:
                raise InvalidParameterError("Parameter {} not in paramter schema".format(key))
            self._validate_parameter_type(key, value, parameter_schema[key])
        return True

    @staticmethod
    def _validate_parameter_type(key, value, type_):
        if not isinstance(value, type_):
            raise InvalidParameterError("Parameter {} has invalid type, expecting {}.".format(key, type_))
        return True
