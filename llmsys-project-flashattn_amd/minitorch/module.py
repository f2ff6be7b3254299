"""Module / Parameter tree (reference ``minitorch/module.py``)."""
from __future__ import annotations

from typing import Any, Dict, Optional, Sequence, Tuple


class Module:
    _modules: Dict[str, "Module"]
    _parameters: Dict[str, "Parameter"]
    training: bool

    def __init__(self) -> None:
        self.__dict__["_modules"] = {}
        self.__dict__["_parameters"] = {}
        self.__dict__["training"] = True

    def modules(self) -> Sequence["Module"]:
        return list(self.__dict__["_modules"].values())

    def train(self) -> None:
        for m in self.modules():
            m.train()
        self.__dict__["training"] = True

    def eval(self) -> None:
        for m in self.modules():
            m.eval()
        self.__dict__["training"] = False

    def named_parameters(self) -> Sequence[Tuple[str, "Parameter"]]:
        out = list(self.__dict__["_parameters"].items())
        for name, m in self.__dict__["_modules"].items():
            out.extend((f"{name}.{k}", v) for k, v in m.named_parameters())
        return out

    def parameters(self) -> Sequence["Parameter"]:
        return [p for _, p in self.named_parameters()]

    def add_parameter(self, k: str, v: Any) -> "Parameter":
        val = Parameter(v, k)
        self.__dict__["_parameters"][k] = val
        return val

    def __setattr__(self, key: str, val: Any) -> None:
        if isinstance(val, Parameter):
            self.__dict__["_parameters"][key] = val
        elif isinstance(val, Module):
            self.__dict__["_modules"][key] = val
        else:
            super().__setattr__(key, val)

    def __getattr__(self, key: str) -> Any:
        d = self.__dict__
        if key in d.get("_parameters", {}):
            return d["_parameters"][key]
        if key in d.get("_modules", {}):
            return d["_modules"][key]
        return None

    def __call__(self, *args: Any, **kwargs: Any) -> Any:
        return self.forward(*args, **kwargs)

    def __repr__(self) -> str:
        lines = [f"({k}): " + repr(m).replace("\n", "\n  ") for k, m in self.__dict__["_modules"].items()]
        body = ("\n  " + "\n  ".join(lines) + "\n") if lines else ""
        return f"{self.__class__.__name__}({body})"


class Parameter:
    def __init__(self, x: Any, name: Optional[str] = None) -> None:
        self.value = x
        self.name = name
        if hasattr(x, "requires_grad_"):
            self.value.requires_grad_(True)
            if self.name:
                self.value.name = self.name

    def update(self, x: Any) -> None:
        self.value = x
        if hasattr(x, "requires_grad_"):
            self.value.requires_grad_(True)
            if self.name:
                self.value.name = self.name

    def __repr__(self) -> str:
        return repr(self.value)

    def __str__(self) -> str:
        return str(self.value)
