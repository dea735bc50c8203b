"""Build hook: `pip install .` / `python setup.py build_ext` compile the gfx950 HIP extension
in-tree via pyrecover_amd/_build.py (hipcc --offload-arch=gfx950), then package it."""
from setuptools import setup
from setuptools.command.build_py import build_py


class BuildWithNative(build_py):
    def run(self):
        import os
        import sys

        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from pyrecover_amd import _build

        _build.build(jobs=min(8, os.cpu_count() or 1))
        super().run()


setup(cmdclass={"build_py": BuildWithNative})
