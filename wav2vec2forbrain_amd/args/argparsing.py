"""Command line -> Experiment — mirrors reference src/args/argparsing.py:14-88: the `experiments`
registry, one --flag per pydantic field of the chosen experiment's args model (bool / list / Literal
parsing as the reference), and get_experiment_from_args() used by run.py."""
from __future__ import annotations

import argparse
import json
import typing
from typing import Any, Literal, Type

from pydantic import BaseModel

from ..experiments.b2t_gru_w2v_conformer_experiment import B2TGruAndW2VConformerExperiment
from ..experiments.b2t_gru_w2v_experiment import B2TGruAndW2VExperiment
from ..experiments.experiment import Experiment
from .base_args import BaseExperimentArgsModel
from .yaml_config import YamlConfig

experiments: dict[str, Type[Experiment]] = {
    "b2p2t_gru+w2v": B2TGruAndW2VExperiment,
    "b2p2t_gru+w2v_conformer": B2TGruAndW2VConformerExperiment,
}


def str_to_bool(value):
    if value.lower() in ["true", "t"]:
        return True
    if value.lower() in ["false", "f"]:
        return False
    if value.lower() in ["none", "n"]:
        return None
    raise argparse.ArgumentTypeError("Invalid boolean value: {}".format(value))


def str_to_list(value):
    parsed = json.loads(value)
    if not isinstance(parsed, list):
        raise argparse.ArgumentTypeError("Invalid list value: {}".format(value))
    return parsed


def _strip_optional(tp):
    if typing.get_origin(tp) is typing.Union:
        args = [a for a in typing.get_args(tp) if a is not type(None)]
        if len(args) == 1:
            return args[0]
    return tp


def _type_args(annotation) -> dict[str, Any]:
    tp = _strip_optional(annotation)
    origin = typing.get_origin(tp)
    if origin is Literal:
        return {"type": str, "choices": typing.get_args(tp)}
    if tp is bool:
        return {"type": str_to_bool}
    if origin is list or tp is list:
        return {"type": str_to_list}
    if tp in (int, float, str):
        return {"type": tp}
    return {"type": str}


def _parser_from_model(parser: argparse.ArgumentParser, model: Type[BaseModel]):
    """One --name per field (pydantic v2 model_fields; the reference reads v1 __fields__)."""
    for name, field in model.model_fields.items():
        default = field.get_default(call_default_factory=True)
        parser.add_argument(f"--{name}", dest=name, default=default, help=field.description,
                            **_type_args(field.annotation))
    return parser


def _create_arg_parser(argv=None):
    base = _parser_from_model(argparse.ArgumentParser(), BaseExperimentArgsModel)
    base_args, _ = base.parse_known_args(argv)
    model = experiments[base_args.experiment_type].get_args_model()
    return _parser_from_model(argparse.ArgumentParser(description="Machine Learning Experiment Configuration"), model)


def get_experiment_from_args(argv=None, config_path: str = "config.yaml") -> Experiment:
    args = _create_arg_parser(argv).parse_args(argv)
    yaml_config = YamlConfig(config_path)
    return experiments[args.experiment_type](vars(args), yaml_config.config)
