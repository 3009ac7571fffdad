"""Scheduler configuration: tiers of plugins (pkg/scheduler/conf/scheduler_conf.go:20-50).

The default configuration is the reference's (pkg/scheduler/util.go:30-40).
"""
from dataclasses import dataclass, field
from typing import List

import yaml

from . import _abi

DEFAULT_SCHEDULER_CONF = """
actions: "allocate, backfill"
tiers:
- plugins:
  - name: priority
  - name: gang
- plugins:
  - name: drf
  - name: predicates
  - name: proportion
"""


@dataclass
class PluginOption:
    name: str
    job_order_disabled: bool = False
    job_ready_disabled: bool = False
    task_order_disabled: bool = False
    preemptable_disabled: bool = False
    reclaimable_disabled: bool = False
    queue_order_disabled: bool = False
    predicate_disabled: bool = False

    _YAML = {"disableJobOrder": "job_order_disabled", "disableJobReady": "job_ready_disabled",
             "disableTaskOrder": "task_order_disabled", "disablePreemptable": "preemptable_disabled",
             "disableReclaimable": "reclaimable_disabled", "disableQueueOrder": "queue_order_disabled",
             "disablePredicate": "predicate_disabled"}

    @staticmethod
    def from_dict(d):
        o = PluginOption(name=d["name"])
        for k, attr in PluginOption._YAML.items():
            setattr(o, attr, bool(d.get(k, False)))
        return o

    def flags(self):
        f = 0
        f |= _abi.DISABLE_JOB_ORDER if self.job_order_disabled else 0
        f |= _abi.DISABLE_JOB_READY if self.job_ready_disabled else 0
        f |= _abi.DISABLE_TASK_ORDER if self.task_order_disabled else 0
        f |= _abi.DISABLE_PREEMPTABLE if self.preemptable_disabled else 0
        f |= _abi.DISABLE_RECLAIMABLE if self.reclaimable_disabled else 0
        f |= _abi.DISABLE_QUEUE_ORDER if self.queue_order_disabled else 0
        f |= _abi.DISABLE_PREDICATE if self.predicate_disabled else 0
        return f


@dataclass
class Tier:
    plugins: List[PluginOption] = field(default_factory=list)


def tiers_from_list(tiers):
    """Fixture form: [[{name, disable*...}, ...], ...] or [{plugins: [...]}, ...]."""
    out = []
    for t in tiers:
        plugins = t["plugins"] if isinstance(t, dict) else t
        out.append(Tier([PluginOption.from_dict(p) for p in plugins]))
    return out


def load_scheduler_conf(conf_str=DEFAULT_SCHEDULER_CONF):
    """pkg/scheduler/util.go:42-64: returns (action names, tiers)."""
    c = yaml.safe_load(conf_str) or {}
    actions = [a.strip() for a in str(c.get("actions", "")).split(",") if a.strip()]
    return actions, tiers_from_list(c.get("tiers") or [])
