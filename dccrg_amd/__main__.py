from .build import build

print(build(force=True, verbose=True))
