"""Exception types of the h2o-py client (reference: ``h2o-py/h2o/exceptions.py``): user-facing errors are
``H2OSoftError`` subclasses (printed without a stack trace by the reference's excepthook), server-side failures are
``H2OResponseError`` / ``H2OServerError``."""


class H2OError(Exception):
    """Base class of every h2o client error."""


class H2OSoftError(H2OError):
    """An error in how the API was called (bad argument, bad state), not a bug."""


class H2OValueError(H2OSoftError, ValueError):
    """An argument has an invalid value."""

    def __init__(self, message, var_name=None, skip_frames=0):
        super().__init__(message)
        self.var_name = var_name
        self.skip_frames = skip_frames


class H2OTypeError(H2OSoftError, TypeError):
    """An argument has an invalid type."""

    def __init__(self, var_name=None, var_value=None, var_type_name=None, exp_type_name=None, message=None,
                 skip_frames=0):
        msg = message or (f"Argument `{var_name}` should be {exp_type_name}, got {var_type_name} {var_value!r}"
                          if var_name is not None else "invalid type")
        super().__init__(msg)
        self.var_name, self.var_value = var_name, var_value
        self.skip_frames = skip_frames


class H2OStartupError(H2OSoftError):
    """The server could not be started."""


class H2OConnectionError(H2OSoftError):
    """No connection to the server could be made."""


class H2OResponseError(H2OError, EnvironmentError):
    """The server answered with an error (4xx)."""


class H2OServerError(H2OError):
    """The server failed (5xx) or answered with something that cannot be parsed."""

    def __init__(self, message, stacktrace=None):
        super().__init__(message)
        self.stacktrace = stacktrace


class H2OJobCancelled(H2OError):
    """A job was cancelled by the user."""


class H2ODeprecationWarning(DeprecationWarning):
    """A deprecated API was used."""
