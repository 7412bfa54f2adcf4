"""Name -> class registry with the reference's semantics (utils/registry.py:23-92):
`register()` as decorator or call, duplicate names raise AssertionError,
unknown names raise KeyError."""


class Registry:
    def __init__(self, name):
        self._name = name
        self._items = {}

    def _add(self, key, obj):
        assert key not in self._items, f"An object named '{key}' was already registered in '{self._name}' registry!"
        self._items[key] = obj

    def register(self, obj=None):
        if obj is not None:
            self._add(obj.__name__, obj)
            return obj

        def deco(target):
            self._add(target.__name__, target)
            return target
        return deco

    def get(self, name):
        if name not in self._items:
            raise KeyError(f"No object named '{name}' found in '{self._name}' registry!")
        return self._items[name]

    def __contains__(self, name):
        return name in self._items

    def __iter__(self):
        return iter(sorted(self._items))
