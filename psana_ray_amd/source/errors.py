"""Source errors (a module of their own: the psana adapter raises them and ``source`` re-exports them)."""


class NoSourceError(RuntimeError):
    """No event source exists for ``(exp, run, detector_name)`` (the reference fails at import
    when psana_wrapper is missing, psana_ray/producer.py:11)."""
