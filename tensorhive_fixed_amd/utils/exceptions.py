"""Domain exceptions (reference ``core/utils/exceptions.py``, ``exceptions/*.py``)."""


class ConfigurationException(Exception):
    pass


class ForbiddenException(Exception):
    pass


class InvalidRequestException(Exception):
    pass


class TransportError(Exception):
    """A node could not be reached / a remote command could not be run."""
