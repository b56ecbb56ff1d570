"""ConfigDict: `ml_collections.ConfigDict` when installed, else a minimal
attribute-dict with the subset of its API the configs and pipelines use
(attribute get/set, nested dicts, update, to_dict, copy_and_resolve_references)."""
from __future__ import annotations

try:  # pragma: no cover - depends on the environment
    from ml_collections import ConfigDict  # type: ignore
except ImportError:  # ml_collections is absent in this image
    import copy

    class ConfigDict(dict):
        def __init__(self, initial=None, **kwargs):
            super().__init__()
            for k, v in dict(initial or {}, **kwargs).items():
                self[k] = v

        def __setitem__(self, k, v):
            if isinstance(v, dict) and not isinstance(v, ConfigDict):
                v = ConfigDict(v)
            super().__setitem__(k, v)

        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError as e:
                raise AttributeError(k) from e

        def __setattr__(self, k, v):
            self[k] = v

        def __delattr__(self, k):
            del self[k]

        def update(self, *args, **kwargs):
            for k, v in dict(*args, **kwargs).items():
                self[k] = v

        def to_dict(self):
            return {k: (v.to_dict() if isinstance(v, ConfigDict) else v) for k, v in self.items()}

        def copy_and_resolve_references(self):
            return copy.deepcopy(self)

        def __deepcopy__(self, memo):
            return ConfigDict({k: copy.deepcopy(v, memo) for k, v in self.items()})
