"""HCL2 parsing and evaluation for ``main.tf`` files."""
from .evaluate import Configuration, Context, EvaluationError
from .parser import Block, Body, HCLSyntaxError, parse, parse_expression, parse_file

__all__ = ["Configuration", "Context", "EvaluationError", "Block", "Body", "HCLSyntaxError",
           "parse", "parse_expression", "parse_file"]
