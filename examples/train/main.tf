# Config 2 of BASELINE.json: PyTorch-ROCm training on MI355X GPUs of this node, with the
# workdir staged into HBM and preemption-safe checkpoints (SIGTERM -> save -> respawn ->
# resume).  `leo preempt <id>` (or `tpi destroy`) exercises the recovery path.
#   tpi apply -auto-approve && leo read --cloud mi355x --follow <id> && tpi destroy -auto-approve
terraform {
  required_providers {
    iterative = { source = "iterative/iterative" }
  }
}

variable "gpus" {
  default = 1
}

resource "iterative_task" "train" {
  name        = "train-example"
  cloud       = "mi355x"
  machine     = "m+mi355x"
  parallelism = var.gpus
  timeout     = 3600
  environment = {
    TPI_FRAMEWORK_ROOT = abspath("../..")
  }
  storage {
    workdir = "."
    output  = "results"
  }
  script = <<-END
    #!/bin/sh
    exec python3 train.py --stage --steps 200 --ckpt-every 50
  END
}

output "logs" {
  value = try(join("\n", iterative_task.train.logs), "")
}
