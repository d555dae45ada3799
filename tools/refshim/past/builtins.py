basestring = str
xrange = range
