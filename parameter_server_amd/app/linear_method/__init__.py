"""Linear-method apps: async SGD (FTRL / AdaGrad / SGD), Darlin BCD, evaluation.

Reference factory: ``LM::createApp`` picks the app by role and config
(src/app/linear_method/linear.cc:8-33).
"""
from __future__ import annotations


def create_linear_app(lm, role: str, name: str = "app"):
    if lm.has("validation_data") and lm.has("model_input") and not lm.has("training_data"):
        from .model_evaluation import ModelEvaluation

        return ModelEvaluation(lm, name) if role == "SCHEDULER" else _Idle(name)
    if lm.has("darlin"):
        from .darlin import DarlinScheduler, DarlinServer, DarlinWorker

        cls = {"SCHEDULER": DarlinScheduler, "SERVER": DarlinServer, "WORKER": DarlinWorker}[role]
        return cls(lm, name)
    if lm.has("async_sgd"):
        from .async_sgd import AsyncSGDScheduler, AsyncSGDServer, AsyncSGDWorker

        cls = {"SCHEDULER": AsyncSGDScheduler, "SERVER": AsyncSGDServer,
               "WORKER": AsyncSGDWorker}[role]
        return cls(lm, name)
    raise ValueError("linear_method config needs async_sgd, darlin or validation_data+model_input")


def _Idle(name):
    from ...system.customer import App

    return App(name)
