// Fixture: a formatter and the fetch the realm replaces with its stand-in.
export function formatWatts(w: number): string {
  return `${w.toFixed(1)} W`;
}

export async function fetchGpuMetrics(): Promise<null> {
  return null;
}
