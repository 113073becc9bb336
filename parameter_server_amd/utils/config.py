"""Typed app configuration from protobuf text format.

The reference configures every app through text-format protos
(``AppConfig{linear_method: LM.Config}``, src/app/main/proto/app.proto,
src/app/linear_method/proto/linear.proto, src/data/proto/data.proto,
src/learner/proto/{sgd,bcd}.proto, src/parameter/proto/param.proto,
src/filter/proto/filter.proto). The text is tokenised by the C++ parser in
``_pscore`` (csrc/core/textproto.cc); this module maps the tree onto typed
messages with the same field names, enum names and proto2 defaults, so the
reference's ``example/linear/**/*.conf`` files load unchanged (including
``[PS.LM.delta_init_value]``-style extension fields).
"""
from __future__ import annotations

import copy
from typing import Any

from ..ops.native import core


class F:
    """Field spec: kind in {int,float,bool,str,enum,msg}; msg = nested schema class."""

    def __init__(self, kind, default=None, repeated=False, enum=None, msg=None, required=False):
        self.kind, self.default, self.repeated = kind, default, repeated
        self.enum, self.msg, self.required = enum, msg, required


class Message:
    FIELDS: dict[str, F] = {}

    def __init__(self, **kw):
        object.__setattr__(self, "_set", {})
        for k, v in kw.items():
            setattr(self, k, v)

    def __getattr__(self, name):
        fields = type(self).FIELDS
        if name not in fields:
            raise AttributeError(f"{type(self).__name__} has no field {name!r}")
        f = fields[name]
        s = object.__getattribute__(self, "_set")
        if name in s:
            return s[name]
        if f.repeated:
            s[name] = []
            return s[name]
        if f.kind == "msg":
            return f.msg()
        return f.default

    def __setattr__(self, name, value):
        if name not in type(self).FIELDS:
            raise AttributeError(f"{type(self).__name__} has no field {name!r}")
        self._set[name] = value

    def has(self, name) -> bool:
        return name in self._set and (not type(self).FIELDS[name].repeated or bool(self._set[name]))

    def mutable(self, name):
        f = type(self).FIELDS[name]
        if name not in self._set:
            self._set[name] = [] if f.repeated else (f.msg() if f.kind == "msg" else f.default)
        return self._set[name]

    def copy(self):
        return copy.deepcopy(self)

    def __eq__(self, other):
        return type(self) is type(other) and self.to_dict() == other.to_dict()

    def to_dict(self) -> dict:
        out = {}
        for k, v in self._set.items():
            if isinstance(v, Message):
                out[k] = v.to_dict()
            elif isinstance(v, list):
                out[k] = [x.to_dict() if isinstance(x, Message) else x for x in v]
            else:
                out[k] = v
        return out

    def __repr__(self):
        return f"{type(self).__name__}({self.to_dict()})"

    # ---------------------------------------------------------------- parse
    @classmethod
    def from_tree(cls, tree) -> "Message":
        m = cls()
        for name, kind, payload in tree:
            if name not in cls.FIELDS:
                raise ValueError(f"{cls.__name__}: unknown field {name!r}")
            f = cls.FIELDS[name]
            if kind == "message":
                if f.kind != "msg":
                    raise ValueError(f"{cls.__name__}.{name}: expected scalar")
                val = f.msg.from_tree(payload)
            else:
                val = _convert(f, payload.decode(), f"{cls.__name__}.{name}")
            if f.repeated:
                m.mutable(name).append(val)
            else:
                m._set[name] = val
        return m

    @classmethod
    def parse(cls, text: str) -> "Message":
        return cls.from_tree(core().parse_textproto(text))

    def to_tree(self):
        out = []
        for name, f in type(self).FIELDS.items():
            if name not in self._set:
                continue
            vals = self._set[name] if f.repeated else [self._set[name]]
            for v in vals:
                if isinstance(v, Message):
                    out.append((name, "message", v.to_tree()))
                elif f.kind == "str":
                    out.append((name, "string", str(v).encode()))
                elif f.kind == "bool":
                    out.append((name, "ident", b"true" if v else b"false"))
                elif f.kind == "enum":
                    out.append((name, "ident", str(v).encode()))
                else:
                    out.append((name, "number", repr(v).encode()))
        return out

    def to_text(self) -> str:
        return core().print_textproto(self.to_tree())


def _convert(f: F, text: str, where: str):
    try:
        if f.kind == "int":
            return int(text, 0) if text.lower().startswith(("0x", "-0x")) else int(float(text)) if "e" in text.lower() else int(text)
        if f.kind == "float":
            return float(text)
        if f.kind == "bool":
            t = text.lower()
            if t in ("true", "1", "t"):
                return True
            if t in ("false", "0", "f"):
                return False
            raise ValueError(text)
        if f.kind == "enum":
            if text not in f.enum:
                raise ValueError(f"{text!r} not in {f.enum}")
            return text
        return text
    except ValueError as e:
        raise ValueError(f"{where}: bad value {text!r}: {e}") from None


# ------------------------------------------------------------------- schemas
class PbRange(Message):
    FIELDS = {"begin": F("int", 0), "end": F("int", 0)}


class HDFSConfig(Message):
    FIELDS = {"home": F("str", ""), "ugi": F("str", ""), "namenode": F("str", "")}


class DataConfig(Message):
    FIELDS = {
        "format": F("enum", "TEXT", enum=("BIN", "PROTO", "TEXT"), required=True),
        "text": F("enum", "LIBSVM", enum=("DENSE", "SPARSE", "SPARSE_BINARY", "ADFEA", "LIBSVM",
                                          "TERAFEA", "VW", "CRITEO")),
        "file": F("str", repeated=True),
        "hdfs": F("msg", msg=HDFSConfig),
        "range": F("msg", msg=PbRange),
        "ignore_feature_group": F("bool", False),
        "max_num_files_per_worker": F("int", -1),
        "max_num_lines_per_file": F("int", -1),
    }


class LossConfig(Message):
    FIELDS = {"type": F("enum", "LOGIT", enum=("SQUARE", "LOGIT", "HINGE", "SQUARE_HINGE"))}


class PenaltyConfig(Message):
    FIELDS = {"type": F("enum", "L1", enum=("L1", "L2")), "lambda": F("float", repeated=True)}


class LearningRateConfig(Message):
    FIELDS = {"type": F("enum", "CONSTANT", enum=("CONSTANT", "DECAY")),
              "alpha": F("float", 1.0), "beta": F("float", 0.0)}


class SGDConfig(Message):
    FIELDS = {
        "algo": F("enum", "FTRL", enum=("STANDARD", "FTRL", "ADAGRAD"), required=True),
        "minibatch": F("int", 1000),
        "data_buf": F("int", 1000),
        "ada_grad": F("bool", True),
        "max_delay": F("int", 0),
        "num_data_pass": F("int", 1),
        "report_interval": F("int", 1),
        "tail_feature_freq": F("int", 0),
        "countmin_n": F("float", 1e8),
        "countmin_k": F("int", 2),
        "fixing_float_by_nbytes": F("int", 0),
    }


class ParameterInitConfig(Message):
    FIELDS = {"type": F("enum", "ZERO", enum=("ZERO", "CONSTANT", "GAUSSIAN", "FILE", "CLONE")),
              "constant": F("float", 1.0), "mean": F("float", 0.0), "std": F("float", 1.0),
              "file_name": F("str", "")}


class BCDConfig(Message):
    FIELDS = {
        "feature_block_ratio": F("float", 4.0),
        "random_feature_block_order": F("bool", True),
        "prior_fea_group": F("int", repeated=True),
        "num_iter_for_prior_fea_group": F("int", 5),
        "max_block_delay": F("int", 0),
        "max_pass_of_data": F("int", 10),
        "epsilon": F("float", 1e-4),
        "tail_feature_freq": F("int", 0),
        "countmin_k": F("int", 2),
        "countmin_n_ratio": F("float", 2.0),
        "max_num_parallel_groups_in_preprocessing": F("int", 1000),
        "max_data_buf_size_in_mb": F("int", 1000),
        "local_cache": F("msg", msg=DataConfig),
        "init_w": F("msg", msg=ParameterInitConfig),
        # proto2 extensions from linear.proto:22-32
        "[PS.LM.delta_init_value]": F("float", 1.0),
        "[PS.LM.delta_max_value]": F("float", 5.0),
        "[PS.LM.kkt_filter_threshold_ratio]": F("float", 10.0),
    }

    def ext(self, short: str):
        return getattr(self, f"[PS.LM.{short}]")


class LMConfig(Message):
    FIELDS = {
        "training_data": F("msg", msg=DataConfig),
        "validation_data": F("msg", msg=DataConfig),
        "model_output": F("msg", msg=DataConfig),
        "model_input": F("msg", msg=DataConfig),
        "loss": F("msg", msg=LossConfig),
        "penalty": F("msg", msg=PenaltyConfig),
        "learning_rate": F("msg", msg=LearningRateConfig),
        "async_sgd": F("msg", msg=SGDConfig),
        "darlin": F("msg", msg=BCDConfig),
    }


class WideDeepConfig(Message):
    """Embedding-table model (BASELINE config 5); new, not in the reference."""

    FIELDS = {
        "training_data": F("msg", msg=DataConfig),
        "num_features": F("int", 10 ** 9),
        "embedding_dim": F("int", 128),
        "hidden": F("int", repeated=True),
        "minibatch": F("int", 4096),
        "learning_rate": F("msg", msg=LearningRateConfig),
        "embedding_dtype": F("enum", "BF16", enum=("FP32", "BF16")),
    }


class AppConfig(Message):
    FIELDS = {"app_name": F("str", ""), "linear_method": F("msg", msg=LMConfig),
              "wide_deep": F("msg", msg=WideDeepConfig)}


def load_app_config(app_file: str | None = None, app_conf: str | None = None) -> AppConfig:
    """Reference semantics: the node config is the content of --app_file followed by
    --app_conf (src/ps.h:18-22, postoffice.cc:61-70)."""
    text = ""
    if app_file:
        with open(app_file) as f:
            text += f.read() + "\n"
    if app_conf:
        text += app_conf
    return AppConfig.parse(text)


def lm_to_sparse_lr(lm: LMConfig, **overrides: Any):
    """Map an LM.Config (async_sgd) onto the GPU trainer config."""
    from ..models.sparse_lr import SparseLRConfig

    sgd = lm.async_sgd
    lam = list(lm.penalty.__getattr__("lambda")) or [0.0]
    if lm.penalty.type == "L1":
        l1, l2 = lam[0], (lam[1] if len(lam) > 1 else 0.0)
    else:
        l1, l2 = 0.0, lam[0]
    if sgd.algo == "FTRL":
        algo = "ftrl"
    elif sgd.algo == "ADAGRAD" or sgd.ada_grad:
        # reference async_sgd.h:136-140 picks the entry type with an inverted test;
        # here ada_grad: true means AdaGrad, as the flag name says.
        algo = "adagrad"
    else:
        algo = "sgd"
    kw = dict(minibatch=sgd.minibatch, loss=lm.loss.type.lower(), algo=algo,
              lr_type=lm.learning_rate.type.lower(), alpha=lm.learning_rate.alpha,
              beta=lm.learning_rate.beta, l1=l1, l2=l2,
              tail_feature_freq=sgd.tail_feature_freq, countmin_n=sgd.countmin_n,
              countmin_k=sgd.countmin_k, fixing_float_bytes=sgd.fixing_float_by_nbytes,
              consistency=f"ssp:{sgd.max_delay}" if sgd.max_delay > 0 else "bsp")
    kw.update(overrides)
    return SparseLRConfig(**kw)
