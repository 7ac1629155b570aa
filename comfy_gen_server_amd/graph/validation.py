"""Prompt validation (parity: ``execution.py:603-918``; C08).

Checks required inputs, link arity, linked RETURN_TYPES vs declared input type ("*" matches
anything), coerces INT/FLOAT/STRING, min/max, combo membership (skipped for inputs handled by a
node's ``VALIDATE_INPUTS``), runs ``VALIDATE_INPUTS`` through the list mapper, and aggregates
per-node errors with ``dependent_outputs``. Extra vs the reference: links to missing nodes and
unknown class_types are reported as validation errors instead of raising KeyError.
"""
from __future__ import annotations

import inspect
import logging
import sys
import traceback

from .executor import get_input_data, map_node_over_list, full_type_name


def _registry():
    from . import registry
    return registry


def _err(typ, message, details, **extra):
    return {"type": typ, "message": message, "details": details, "extra_info": extra}


def validate_inputs(prompt, item, validated):
    nodes = _registry().NODE_CLASS_MAPPINGS
    uid = item
    if uid in validated:
        return validated[uid]
    node = prompt[uid]
    inputs = node["inputs"]
    class_type = node["class_type"]
    if class_type not in nodes:
        ret = (False, [_err("invalid_prompt", f"Cannot execute because node {class_type} does not exist.",
                            f"Node ID '#{uid}'")], uid)
        validated[uid] = ret
        return ret
    obj_class = nodes[class_type]
    class_inputs = obj_class.INPUT_TYPES()
    required = class_inputs.get("required", {})
    errors = []
    valid = True
    vfi = []
    if hasattr(obj_class, "VALIDATE_INPUTS"):
        vfi = inspect.getfullargspec(obj_class.VALIDATE_INPUTS).args
    info = None
    val = None
    for x, info in required.items():
        if x not in inputs:
            errors.append(_err("required_input_missing", "Required input is missing", f"{x}", input_name=x))
            continue
        val = inputs[x]
        type_input = info[0]
        if isinstance(val, list):
            if len(val) != 2:
                errors.append(_err("bad_linked_input", "Bad linked input, must be a length-2 list of [node_id, slot_index]",
                                   f"{x}", input_name=x, input_config=info, received_value=val))
                continue
            o_id = val[0]
            if o_id not in prompt or prompt[o_id].get("class_type") not in nodes:
                errors.append(_err("bad_linked_input", "Linked node does not exist", f"{x}: {o_id}", input_name=x,
                                   linked_node=val))
                continue
            r = nodes[prompt[o_id]["class_type"]].RETURN_TYPES
            if not isinstance(val[1], int) or val[1] >= len(r):
                errors.append(_err("bad_linked_input", "Linked output slot out of range", f"{x}: {val}", input_name=x,
                                   linked_node=val))
                continue
            received = r[val[1]]
            if received != type_input and type_input != "*" and received != "*":
                errors.append(_err("return_type_mismatch", "Return type mismatch between linked nodes",
                                   f"{x}, {received} != {type_input}", input_name=x, input_config=info,
                                   received_type=received, linked_node=val))
                continue
            try:
                rr = validate_inputs(prompt, o_id, validated)
                if rr[0] is False:
                    valid = False
                    continue
            except Exception as ex:
                typ, _, tb = sys.exc_info()
                valid = False
                validated[o_id] = (False, [_err("exception_during_inner_validation", "Exception when validating inner node",
                                                str(ex), input_name=x, input_config=info, exception_message=str(ex),
                                                exception_type=full_type_name(typ), traceback=traceback.format_tb(tb),
                                                linked_node=val)], o_id)
                continue
        else:
            try:
                if type_input == "INT":
                    val = int(val)
                    inputs[x] = val
                elif type_input == "FLOAT":
                    val = float(val)
                    inputs[x] = val
                elif type_input == "STRING":
                    val = str(val)
                    inputs[x] = val
                elif type_input == "BOOLEAN":
                    val = bool(val)
                    inputs[x] = val
            except Exception as ex:
                errors.append(_err("invalid_input_type", f"Failed to convert an input value to a {type_input} value",
                                   f"{x}, {val}, {ex}", input_name=x, input_config=info, received_value=val,
                                   exception_message=str(ex)))
                continue
            if len(info) > 1 and isinstance(info[1], dict):
                if "min" in info[1] and val < info[1]["min"]:
                    errors.append(_err("value_smaller_than_min", f"Value {val} smaller than min of {info[1]['min']}",
                                       f"{x}", input_name=x, input_config=info, received_value=val))
                    continue
                if "max" in info[1] and val > info[1]["max"]:
                    errors.append(_err("value_bigger_than_max", f"Value {val} bigger than max of {info[1]['max']}",
                                       f"{x}", input_name=x, input_config=info, received_value=val))
                    continue
            if x not in vfi and isinstance(type_input, list) and val not in type_input:
                cfg = info
                if len(type_input) > 20:
                    li = f"(list of length {len(type_input)})"
                    cfg = None
                else:
                    li = str(type_input)
                errors.append(_err("value_not_in_list", "Value not in list", f"{x}: '{val}' not in {li}",
                                   input_name=x, input_config=cfg, received_value=val))
                continue
    if vfi:
        ida = get_input_data(inputs, obj_class, uid)
        filt = {k: v for k, v in ida.items() if k in vfi}
        ret = map_node_over_list(obj_class, filt, "VALIDATE_INPUTS")
        for x in filt:
            for r in ret:
                if r is not True:
                    d = f"{x}" + (f" - {r}" if r is not False else "")
                    errors.append(_err("custom_validation_failed", "Custom validation failed for node", d,
                                       input_name=x, input_config=info, received_value=val))
    ret = (False, errors, uid) if (errors or valid is not True) else (True, [], uid)
    validated[uid] = ret
    return ret


def validate_prompt(prompt):
    nodes = _registry().NODE_CLASS_MAPPINGS
    outputs = set()
    for x, node in prompt.items():
        if x == "outputs":
            continue
        if not isinstance(node, dict) or "class_type" not in node:
            return (False, _err("invalid_prompt", "Cannot execute because a node is missing the class_type property.",
                                f"Node ID '#{x}'"), [], [])
        cls = nodes.get(node["class_type"])
        if cls is None:
            return (False, _err("invalid_prompt", f"Cannot execute because node {node['class_type']} does not exist.",
                                f"Node ID '#{x}'"), [], [])
        if getattr(cls, "OUTPUT_NODE", False) is True:
            outputs.add(x)
    if not outputs:
        return (False, _err("prompt_no_outputs", "Prompt has no outputs", ""), [], [])
    good, errors, node_errors, validated = set(), [], {}, {}
    for o in sorted(outputs):
        try:
            m = validate_inputs(prompt, o, validated)
            valid, reasons = m[0], m[1]
        except Exception as ex:
            typ, _, tb = sys.exc_info()
            valid = False
            reasons = [_err("exception_during_validation", "Exception when validating node", str(ex),
                            exception_type=full_type_name(typ), traceback=traceback.format_tb(tb))]
            validated[o] = (False, reasons, o)
        if valid is True:
            good.add(o)
        else:
            logging.error("Failed to validate prompt for output %s:", o)
            errors.append((o, reasons))
            for nid, res in validated.items():
                if res[0] is not True and res[1]:
                    if nid not in node_errors:
                        node_errors[nid] = {"errors": res[1], "dependent_outputs": [],
                                            "class_type": prompt[nid]["class_type"]}
                    node_errors[nid]["dependent_outputs"].append(o)
    if not good:
        lines = "\n".join(f"{e['message']}: {e['details']}" for _, es in errors for e in es)
        return (False, _err("prompt_outputs_failed_validation", "Prompt outputs failed validation", lines),
                list(good), node_errors)
    return (True, None, list(good), node_errors)
