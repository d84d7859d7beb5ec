{{ $t := .metadata.creationTimestamp }}
conditions:
- lastTransitionTime: {{ $t }}
  status: "True"
  type: PodScheduled
- lastTransitionTime: {{ $t }}
  status: "True"
  type: Ready
{{ range .spec.readinessGates }}
- lastTransitionTime: {{ $t }}
  status: "True"
  type: {{ .conditionType }}
{{ end }}
containerStatuses:
{{ range .spec.containers }}
- image: {{ .image }}
  name: {{ .name }}
  ready: true
  restartCount: 0
  started: true
  state:
    running:
      startedAt: {{ $t }}
{{ end }}
{{ with .status }}
hostIP: {{ with .hostIP }}{{ . }}{{ else }}{{ NodeIP }}{{ end }}
podIP: {{ with .podIP }}{{ . }}{{ else }}{{ PodIP }}{{ end }}
{{ end }}
phase: Running
qosClass: BestEffort
startTime: {{ $t }}
