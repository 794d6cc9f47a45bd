# Config 1 of BASELINE.json: hello world on the CPU of this node.
#   tpi init && tpi apply -auto-approve && tpi refresh && tpi output logs && tpi destroy -auto-approve
terraform {
  required_providers {
    iterative = { source = "iterative/iterative" }
  }
}

resource "iterative_task" "hello" {
  cloud   = "local"
  machine = "s"
  storage {
    workdir = "."
    output  = "results"
  }
  script = <<-END
    #!/bin/sh
    mkdir -p results
    echo "hello from $TPI_MACHINE_IDENTITY" | tee results/hello.txt
  END
}

output "logs" {
  value = try(join("\n", iterative_task.hello.logs), "")
}
