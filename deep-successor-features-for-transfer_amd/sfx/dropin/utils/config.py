"""INI config files whose values are Python literals (the format of the reference's configs/).

``parse_config_file(name)`` looks for ``configs/<name>`` next to the running script first, then
in the current directory, then under $SFX_CONFIG_DIR.
"""
from __future__ import annotations

import configparser
import os
import sys
from ast import literal_eval

global_settings = {}


def _candidates(name):
    main = getattr(sys.modules.get("__main__"), "__file__", None)
    dirs = []
    if main:
        dirs.append(os.path.join(os.path.dirname(os.path.abspath(main)), "configs"))
    dirs.append(os.path.join(os.getcwd(), "configs"))
    if os.environ.get("SFX_CONFIG_DIR"):
        dirs.append(os.environ["SFX_CONFIG_DIR"])
    return [os.path.join(d, name) for d in dirs]


def parse_config_file(name):
    global global_settings
    path = next((p for p in _candidates(name) if os.path.exists(p)), None)
    if path is None:
        raise FileNotFoundError(f"config {name!r} not found in {_candidates(name)}")
    parser = configparser.RawConfigParser()
    parser.optionxform = str
    parser.read(path)
    global_settings = {sec: {k: literal_eval(v) for k, v in parser.items(sec)} for sec in parser.sections()}
    return global_settings


def check_settings():
    if not global_settings:
        raise Exception("Global settings is not initialized")


def use_torch():
    check_settings()
    return global_settings.get("GENERAL", {}).get("use_torch")


def use_logger():
    check_settings()
    return global_settings.get("GENERAL", {}).get("use_torch")
