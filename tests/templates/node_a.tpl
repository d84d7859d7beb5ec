{{ with .status }}
addresses:
- address: {{ NodeIP }}
  type: InternalIP
- address: kwok-node
  type: Hostname
allocatable:
{{ with .allocatable }}
{{ YAML . 1 }}
{{ else }}
  cpu: "32"
  memory: 256Gi
  pods: "110"
{{ end }}
capacity: {cpu: "32", memory: 256Gi, pods: "110"}
nodeInfo:
  architecture: {{ with .nodeInfo.architecture }}{{ . }}{{ else }}amd64{{ end }}
  kubeletVersion: v1.26.0-kwok
  operatingSystem: linux
phase: Running
{{ end }}
