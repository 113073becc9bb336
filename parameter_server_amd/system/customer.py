"""Customers (named distributed objects) and Apps.

Reference: a ``Customer`` is a named RPC endpoint; the same name on different
nodes is the logical peer. It owns an Executor and implements ``process(msg)``;
``slice`` splits a message for a node group (src/system/customer.h:12-58).
``App`` adds ``init``/``run`` and a factory from the text config
(src/system/app.h, src/app/main/main.cc:15-30).
"""
from __future__ import annotations

from .executor import Executor
from .message import Message, slice_key_ordered
from .postoffice import Postoffice


class Customer:
    def __init__(self, name: str, parent: str | None = None, po: Postoffice | None = None):
        self.name = name
        self.parent = parent
        self.po = po or Postoffice.instance()
        if name in self.po.yp.customers:
            raise ValueError(f"customer {name!r} already exists on {self.po.my_node.id}")
        self.executor = Executor(self, self.po)
        self.po.yp.customers[name] = self

    # node id helpers
    @property
    def my_node(self):
        return self.po.my_node

    def my_node_id(self) -> str:
        return self.po.my_node.id

    def my_rank(self) -> int:
        return self.po.my_node.rank

    def scheduler_id(self) -> str:
        return self.po.scheduler.id

    def port(self, node_or_group: str):
        r = self.executor.rnode(node_or_group)
        if r is None:
            raise KeyError(f"{self.name}: unknown node/group {node_or_group}")
        return r

    def process(self, msg: Message):
        """Handle a request; override."""

    def slice(self, msg: Message, key_ranges):
        """Default: replicate the message to every group member."""
        out = []
        for _ in key_ranges:
            m = msg.copy_header()
            m.key, m.value = msg.key, list(msg.value)
            m.fin_handle, m.recv_handle, m.wait = msg.fin_handle, msg.recv_handle, msg.wait
            out.append(m)
        return out

    def stop(self):
        self.executor.stop()
        self.po.yp.customers.pop(self.name, None)


class KeyOrderedCustomer(Customer):
    def slice(self, msg, key_ranges):
        return slice_key_ordered(msg, key_ranges)


class App(Customer):
    REGISTRY = {}

    def __init__(self, name: str = "app", conf=None, po: Postoffice | None = None):
        super().__init__(name, po=po)
        self.conf = conf

    def init(self):
        pass

    def run(self):
        pass

    @classmethod
    def register(cls, key):
        def deco(factory):
            cls.REGISTRY[key] = factory
            return factory

        return deco

    @staticmethod
    def create(conf_text: str) -> "App":
        """Build this node's app from the text config (reference App::create)."""
        from ..utils.config import AppConfig

        conf = AppConfig.parse(conf_text) if conf_text.strip() else AppConfig()
        po = Postoffice.instance()
        role = po.my_node.role
        if conf.has("linear_method"):
            from ..app.linear_method import create_linear_app

            return create_linear_app(conf.linear_method, role)
        name = conf.app_name
        if name and name in App.REGISTRY:
            return App.REGISTRY[name](conf, role)
        if "__default__" in App.REGISTRY:
            return App.REGISTRY["__default__"](conf, role)
        return App()
