"""Minimal stand-in for the `addict` package (attribute-access dict).

Only used by tests/golden/make_golden.py to import the reference in the
survey container; never shipped, never imported by the product path.
"""


class Dict(dict):
    def __init__(self, *args, **kwargs):
        super().__init__()
        for arg in args:
            if isinstance(arg, dict):
                for k, v in arg.items():
                    self[k] = self._hook(v)
            elif isinstance(arg, tuple) and len(arg) == 2 and not isinstance(arg[0], tuple):
                self[arg[0]] = self._hook(arg[1])
            elif arg is not None:
                for k, v in arg:
                    self[k] = self._hook(v)
        for k, v in kwargs.items():
            self[k] = self._hook(v)

    @classmethod
    def _hook(cls, item):
        if isinstance(item, dict):
            return cls(item)
        if isinstance(item, (list, tuple)):
            return type(item)(cls._hook(e) for e in item)
        return item

    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError:
            raise AttributeError(name)

    def __setattr__(self, name, value):
        self[name] = value

    def __delattr__(self, name):
        del self[name]

    def to_dict(self):
        out = {}
        for k, v in self.items():
            if isinstance(v, Dict):
                v = v.to_dict()
            elif isinstance(v, (list, tuple)):
                v = type(v)(e.to_dict() if isinstance(e, Dict) else e for e in v)
            out[k] = v
        return out

    def copy(self):
        return type(self)(self)

    def __deepcopy__(self, memo):
        import copy as _copy
        other = type(self)()
        memo[id(self)] = other
        for k, v in self.items():
            other[_copy.deepcopy(k, memo)] = _copy.deepcopy(v, memo)
        return other

    def update(self, *args, **kwargs):
        for k, v in dict(*args, **kwargs).items():
            self[k] = self._hook(v)
