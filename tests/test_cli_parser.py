"""``tpi``'s parser: only the named subcommand's parser is built (argparse costs ~10 ms for all
ten on every ``tpi apply``), with the same parse results."""
from terraform_provider_iterative_amd.cli import tf


def test_only_the_named_subcommand_is_built_and_parses_the_same():
    assert tf._command_in(["-chdir", "apply", "plan"]) == "plan"  # -chdir's value is no command
    assert tf._command_in(["-chdir=x", "apply", "-auto-approve"]) == "apply"
    assert tf._command_in(["-version"]) is None
    for argv in (["apply", "-auto-approve", "-var", "a=1"], ["destroy", "-auto-approve"],
                 ["output", "-json", "name"], ["state", "rm", "iterative_task.x"],
                 ["plan", "-destroy"], ["version"]):
        full = vars(tf.build_parser().parse_args(argv))
        only = vars(tf.build_parser(argv[0]).parse_args(argv))
        assert full == only, argv
