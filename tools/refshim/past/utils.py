import numbers


def old_div(a, b):
    """Python-2 division semantics: floor division for two integers."""
    if isinstance(a, numbers.Integral) and isinstance(b, numbers.Integral):
        return a // b
    return a / b
