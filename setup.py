"""Build hook: compiles the gfx950 extension in-tree (psana_ray_amd/_build.py) before packaging."""
from setuptools import setup
from setuptools.command.build_py import build_py


class BuildWithNative(build_py):
    def run(self):
        from psana_ray_amd import _build

        _build.build()
        super().run()


setup(cmdclass={"build_py": BuildWithNative})
