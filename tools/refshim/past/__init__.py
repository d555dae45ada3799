"""Minimal stand-in for the `past` package (python-future), used ONLY to import
the read-only reference hyperopt in the survey container when generating golden
fixtures.  Never shipped, never imported by the product."""
