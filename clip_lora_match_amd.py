"""Import shim: the package lives in `clip-lora-match_amd/` (a directory name
Python cannot import directly). Importing this module loads that directory as
the package `clip_lora_match_amd` and replaces this module in sys.modules, so
`import clip_lora_match_amd.search` etc. resolve inside the package."""
import importlib.util as _ilu
import os as _os
import sys as _sys

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "clip-lora-match_amd")
_spec = _ilu.spec_from_file_location(
    __name__, _os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
