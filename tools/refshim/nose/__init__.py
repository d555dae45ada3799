import unittest
SkipTest = unittest.SkipTest
