def raises(*exc):
    def deco(f):
        def wrapper(*a, **k):
            try:
                f(*a, **k)
            except exc:
                return
            raise AssertionError('did not raise %r' % (exc,))
        wrapper.__name__ = f.__name__
        return wrapper
    return deco


def eq_(a, b, msg=None):
    assert a == b, msg or '%r != %r' % (a, b)
