"""Caching graph executor (parity: ``execution.py:60-600``; C09, C10).

Semantics kept from the reference:
  * demand-driven DFS from output nodes; outputs run in order of fewest un-executed dependencies;
  * cross-prompt output cache keyed by node id, invalidated when the node's inputs change, its
    ``IS_CHANGED`` value changes, or any upstream node was invalidated;
  * node instances persist per (id, class_type) in ``object_storage``;
  * list semantics: ``INPUT_IS_LIST``, ``OUTPUT_IS_LIST``, broadcast-last-element slicing, generator
    flattening; ``{"ui": ..., "result": ...}`` returns; hidden PROMPT / EXTRA_PNGINFO / UNIQUE_ID;
  * per-node error isolation -> ``execution_error`` / ``execution_interrupted`` with formatted
    inputs/outputs; downstream outputs that did not run are dropped from the cache;
  * the fork's top-level ``"outputs": {key: [node_id, slot]}`` map is published to the Yjs doc
    (``server.output_map``) after the producing node runs (``execution.py:334-345``), with values
    JSON-encoded safely (the reference's ``json.dumps(bytes)`` raises — SURVEY §7.6).
Differences: no stray debug prints of tensors on the hot path; per-node wall time
is recorded (``node_timings``) and exported as Prometheus metrics by the server.
"""
from __future__ import annotations

import copy
import inspect
import json
import logging
import sys
import time
import traceback

import torch

from ..runtime import device as dm
from ..utils import telemetry


def _registry():
    from . import registry
    return registry


def get_input_data(inputs, class_def, unique_id, outputs=None, prompt=None, extra_data=None):
    valid = class_def.INPUT_TYPES()
    req = valid.get("required", {})
    opt = valid.get("optional", {})
    out = {}
    outputs = outputs or {}
    for name, val in inputs.items():
        if isinstance(val, list):
            src, idx = val[0], val[1]
            if src not in outputs:
                out[name] = (None,)
                continue
            out[name] = outputs[src][idx]
        elif name in req or name in opt:
            out[name] = [val]
    hidden = valid.get("hidden", {})
    for name, kind in hidden.items():
        if kind == "PROMPT":
            out[name] = [prompt]
        elif kind == "EXTRA_PNGINFO":
            out[name] = [extra_data.get("extra_pnginfo")] if extra_data is not None else (None,)
        elif kind == "UNIQUE_ID":
            out[name] = [unique_id]
    return out


def _flatten_call(fn, kwargs, results):
    r = fn(**kwargs)
    if inspect.isgenerator(r):
        results.extend(list(r))
    else:
        results.append(r)


def map_node_over_list(obj, input_data_all, func, allow_interrupt=False):
    input_is_list = getattr(obj, "INPUT_IS_LIST", False)
    max_len = max((len(v) for v in input_data_all.values()), default=0)
    results = []
    fn = getattr(obj, func)
    if input_is_list:
        if allow_interrupt:
            dm.throw_exception_if_processing_interrupted()
        _flatten_call(fn, input_data_all, results)
    elif max_len == 0:
        if allow_interrupt:
            dm.throw_exception_if_processing_interrupted()
        _flatten_call(fn, {}, results)
    else:
        for i in range(max_len):
            if allow_interrupt:
                dm.throw_exception_if_processing_interrupted()
            sl = {k: v[i if len(v) > i else -1] for k, v in input_data_all.items()}
            _flatten_call(fn, sl, results)
    return results


def get_output_data(obj, input_data_all):
    results, uis = [], []
    for r in map_node_over_list(obj, input_data_all, obj.FUNCTION, allow_interrupt=True):
        if isinstance(r, dict):
            if "ui" in r:
                uis.append(r["ui"])
            if "result" in r:
                results.append(r["result"])
        else:
            results.append(r)
    output = []
    if results:
        is_list = getattr(obj, "OUTPUT_IS_LIST", [False] * len(results[0]))
        for i, il in zip(range(len(results[0])), is_list):
            if il:
                output.append([x for o in results for x in o[i]])
            else:
                output.append([o[i] for o in results])
    ui = {}
    if uis:
        ui = {k: [y for x in uis for y in x[k]] for k in uis[0].keys()}
    return output, ui


def format_value(x):
    if x is None or isinstance(x, (int, float, bool, str)):
        return x
    return str(x)


def full_type_name(klass):
    m = klass.__module__
    return klass.__qualname__ if m == "builtins" else m + "." + klass.__qualname__


def _jsonable(v, total=None):
    """Best-effort JSON for the Yjs output map (tensors -> shape summary, bytes -> size). A batch split over
    the ranks of an SPMD prompt (a LATENT with ``dp_shard``, an IMAGE carrying the shard mark) is described
    as the whole batch -- the value one GPU running the prompt whole would publish -- not as this rank's shard."""
    try:
        json.dumps(v)
        return v
    except TypeError:
        pass
    if isinstance(v, torch.Tensor):
        shape = list(v.shape)
        sh = getattr(v, "_cgs_dp_shard", None)
        if sh is not None and shape:
            shape[0] = int(sh[2])
        elif total is not None and shape:
            shape[0] = int(total)
        return {"tensor": shape, "dtype": str(v.dtype)}
    if isinstance(v, (bytes, bytearray)):
        return {"bytes": len(v)}
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if isinstance(v, dict):
        if "dp_shard" in v:
            off, n, tot = v["dp_shard"]
            return {str(k): _jsonable(x, tot if (torch.is_tensor(x) and x.dim() and x.shape[0] == n) else None)
                    for k, x in v.items() if k != "dp_shard"}
        return {str(k): _jsonable(x) for k, x in v.items()}
    return str(v)


class _NullServer:
    client_id = None
    last_node_id = None
    output_map = None

    def send_sync(self, event, data, sid=None):
        pass

    def queue_updated(self):
        pass

    def broadcast_yjs_updates(self):
        pass


class PromptExecutor:
    def __init__(self, server=None, node_hook=None):
        self.server = server or _NullServer()
        self.node_hook = node_hook      # sched.spmd.SPMD for batch-sharded multi-rank prompts
        self.reset()

    def reset(self):
        self.outputs = {}
        self.object_storage = {}
        self.outputs_ui = {}
        self.status_messages = []
        self.success = True
        self.old_prompt = {}
        self.node_timings = {}

    def add_message(self, event, data, broadcast: bool):
        self.status_messages.append((event, data))
        if self.server.client_id is not None or broadcast:
            self.server.send_sync(event, data, self.server.client_id)

    # -------------------------------------------------------------------------------- recursion
    def _execute_node(self, prompt, unique_id, extra_data, executed, prompt_id):
        nodes = _registry().NODE_CLASS_MAPPINGS
        if unique_id in self.outputs:
            return True, None, None
        inputs = prompt[unique_id]["inputs"]
        class_type = prompt[unique_id]["class_type"]
        class_def = nodes[class_type]
        for name, val in inputs.items():
            if isinstance(val, list) and val[0] not in self.outputs:
                r = self._execute_node(prompt, val[0], extra_data, executed, prompt_id)
                if r[0] is not True:
                    return r
        input_data_all = None
        hook = self.node_hook
        try:
            if hook is not None:
                hook.node_begin()
            input_data_all = get_input_data(inputs, class_def, unique_id, self.outputs, prompt, extra_data)
            if self.server.client_id is not None:
                self.server.last_node_id = unique_id
                self.server.send_sync("executing", {"node": unique_id, "prompt_id": prompt_id}, self.server.client_id)
            obj = self.object_storage.get((unique_id, class_type))
            if obj is None:
                obj = class_def()
                self.object_storage[(unique_id, class_type)] = obj
            t0 = time.perf_counter()
            with telemetry.span(f"node:{class_type}:{unique_id}"):
                telemetry.maybe_fault("node", class_type)
                if hook is None:
                    output_data, output_ui = get_output_data(obj, input_data_all)
                else:   # SPMD (sched/spmd.py): agreement points, unsharding, rank-0 output nodes
                    output_data, output_ui = hook.execute(class_type, class_def, obj, input_data_all,
                                                          get_output_data)
            dt = time.perf_counter() - t0
            self.node_timings[unique_id] = (class_type, dt)
            telemetry.record_node(class_type, dt)
            if output_ui and isinstance(output_ui.get("images"), list):
                telemetry.add("images_saved_total", len(output_ui["images"]))
            self.outputs[unique_id] = output_data
            outmap = prompt.get("outputs") if isinstance(prompt.get("outputs"), dict) else None
            if outmap and getattr(self.server, "output_map", None) is not None:
                for key, src in outmap.items():
                    if isinstance(src, (list, tuple)) and len(src) == 2 and str(src[0]) == str(unique_id):
                        val = output_data[src[1]] if src[1] < len(output_data) else None
                        self.server.output_map.set(key, json.dumps(_jsonable(val)))
                        self.server.broadcast_yjs_updates()
            if output_ui:
                self.outputs_ui[unique_id] = output_ui
                if self.server.client_id is not None:
                    self.server.send_sync("executed", {"node": unique_id, "output": output_ui, "prompt_id": prompt_id},
                                          self.server.client_id)
        except dm.InterruptProcessingException as iex:
            if hook is not None:
                hook.abort()
            logging.info("Processing interrupted")
            return False, {"node_id": unique_id}, iex
        except Exception as ex:
            if hook is not None:
                hook.abort()    # the peers are at this node's pending agreement point
            typ, _, tb = sys.exc_info()
            inputs_fmt = {}
            if input_data_all is not None:
                inputs_fmt = {n: [format_value(x) for x in v] for n, v in input_data_all.items()}
            outputs_fmt = {nid: [[format_value(x) for x in l] for l in no] for nid, no in self.outputs.items()}
            logging.error("!!! Exception during processing !!! %s", ex)
            logging.error(traceback.format_exc())
            return False, {"node_id": unique_id, "exception_message": str(ex), "exception_type": full_type_name(typ),
                           "traceback": traceback.format_tb(tb), "current_inputs": inputs_fmt,
                           "current_outputs": outputs_fmt}, ex
        executed.add(unique_id)
        return True, None, None

    def _will_execute(self, prompt, uid, memo):
        if uid in memo:
            return memo[uid]
        if uid in self.outputs:
            return []
        res = []
        for v in prompt[uid]["inputs"].values():
            if isinstance(v, list) and v[0] not in self.outputs:
                res += self._will_execute(prompt, v[0], memo)
        memo[uid] = res + [uid]
        return memo[uid]

    def _delete_if_changed(self, prompt, uid):
        nodes = _registry().NODE_CLASS_MAPPINGS
        node = prompt[uid]
        class_def = nodes[node["class_type"]]
        inputs = node["inputs"]
        is_changed_old = ""
        is_changed = ""
        to_delete = False
        if hasattr(class_def, "IS_CHANGED"):
            if uid in self.old_prompt and "is_changed" in self.old_prompt[uid]:
                is_changed_old = self.old_prompt[uid]["is_changed"]
            if "is_changed" not in node:
                ida = get_input_data(inputs, class_def, uid, self.outputs)
                try:
                    is_changed = map_node_over_list(class_def, ida, "IS_CHANGED")
                    node["is_changed"] = is_changed
                except Exception:
                    to_delete = True
            else:
                is_changed = node["is_changed"]
        if uid not in self.outputs:
            return True
        if not to_delete:
            if is_changed != is_changed_old or uid not in self.old_prompt:
                to_delete = True
            elif inputs == self.old_prompt[uid]["inputs"]:
                for v in inputs.values():
                    if isinstance(v, list):
                        to_delete = self._delete_if_changed(prompt, v[0]) if v[0] in self.outputs else True
                        if to_delete:
                            break
            else:
                to_delete = True
        if to_delete:
            self.outputs.pop(uid, None)
        return to_delete

    def handle_execution_error(self, prompt_id, prompt, current_outputs, executed, error, ex):
        node_id = error["node_id"]
        class_type = prompt[node_id]["class_type"]
        mes = {"prompt_id": prompt_id, "node_id": node_id, "node_type": class_type, "executed": list(executed)}
        if isinstance(ex, dm.InterruptProcessingException):
            self.add_message("execution_interrupted", mes, broadcast=True)
        else:
            mes.update({k: error[k] for k in ("exception_message", "exception_type", "traceback", "current_inputs",
                                             "current_outputs")})
            self.add_message("execution_error", mes, broadcast=False)
        for o in [o for o in self.outputs if o not in current_outputs and o not in executed]:
            self.old_prompt.pop(o, None)
            self.outputs.pop(o, None)

    def execute(self, prompt, prompt_id, extra_data=None, execute_outputs=()):
        extra_data = extra_data or {}
        dm.interrupt_current_processing(False)
        self.server.client_id = extra_data.get("client_id")
        self.status_messages = []
        self.add_message("execution_start", {"prompt_id": prompt_id}, broadcast=False)
        nodes_in_prompt = {k for k in prompt if k != "outputs"}
        with torch.inference_mode():
            for o in [o for o in self.outputs if o not in nodes_in_prompt]:
                self.outputs.pop(o)
            for o in [o for o in self.object_storage
                      if o[0] not in nodes_in_prompt or prompt[o[0]]["class_type"] != o[1]]:
                self.object_storage.pop(o)
            for x in nodes_in_prompt:
                self._delete_if_changed(prompt, x)
            current_outputs = set(self.outputs.keys())
            for x in [x for x in self.outputs_ui if x not in current_outputs]:
                self.outputs_ui.pop(x)
            dm.cleanup_models(keep_clone_weights_loaded=True)
            self.add_message("execution_cached", {"nodes": list(current_outputs), "prompt_id": prompt_id},
                             broadcast=False)
            executed = set()
            to_execute = [(0, n) for n in execute_outputs]
            while to_execute:
                memo = {}
                to_execute = sorted((len(self._will_execute(prompt, a[-1], memo)), a[-1]) for a in to_execute)
                out_id = to_execute.pop(0)[-1]
                self.success, error, ex = self._execute_node(prompt, out_id, extra_data, executed, prompt_id)
                if self.success is not True:
                    self.handle_execution_error(prompt_id, prompt, current_outputs, executed, error, ex)
                    break
            for x in executed:
                self.old_prompt[x] = copy.deepcopy(prompt[x])
            self.server.last_node_id = None
            if dm._args.get("disable_smart_memory"):
                dm.unload_all_models()
