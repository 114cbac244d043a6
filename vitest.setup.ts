import '@testing-library/jest-dom';

// Node 22+ ships a property-bag `localStorage` global that shadows jsdom's
// Web Storage; install a spec-compliant one so code under test behaves.
if (typeof localStorage !== 'undefined' && typeof localStorage.getItem !== 'function') {
  const store = new Map<string, string>();
  const storage: Storage = {
    getItem: (k: string) => (store.has(k) ? (store.get(k) as string) : null),
    setItem: (k: string, v: string) => void store.set(k, String(v)),
    removeItem: (k: string) => void store.delete(k),
    clear: () => store.clear(),
    key: (i: number) => Array.from(store.keys())[i] ?? null,
    get length() {
      return store.size;
    },
  };
  Object.defineProperty(globalThis, 'localStorage', { value: storage, configurable: true, writable: true });
}
