"""Single source of the release version (the reference injects ``utils.Version`` at link
time, ``Makefile:10``).  ``make release VERSION=x.y.z`` rewrites this file; native
components get the same string through ``-DTPI_VERSION_STRING`` (``_build.py``)."""

__version__ = "0.2.0"
